import os, subprocess, sys, numpy as np
sys.path.insert(0, 'tests')
ROOT = os.getcwd()
import importlib.util
spec = importlib.util.spec_from_file_location("km", "tests/test_gpu_krylov_modes.py")
src = open("tests/test_gpu_krylov_modes.py").read()
i = src.index("_ALT_CHILD = r'''") + len("_ALT_CHILD = r'''"); j = src.index("'''", i)
code = src[i:j].replace('restart=20, maxiter=30', 'restart=21, maxiter=25')
res = {}
for tag, env in [("lag0", {"HH_LAG_RED": "0"}), ("lag1", {"HH_LAG_RED": "1"}), ("lag2", {"HH_LAG_RED": "2"}),
                 ("lag0_alt0", {"HH_LAG_RED": "0", "HH_FUSED_ALT": "0"}), ("lag1_alt0", {"HH_LAG_RED": "1", "HH_FUSED_ALT": "0"}),
                 ("lag0_rows16", {"HH_LAG_RED": "0", "HH_FUSED_ROWS": "16"})]:
    out = f"/tmp/sens_{tag}.npz"
    subprocess.run([sys.executable, "-c", code, ROOT, "1024", "c1", "jacobi", out], env=dict(os.environ, **env), check=True, timeout=240)
    res[tag] = np.load(out)
a = res["lag0"]
for k, v in res.items():
    dx = np.linalg.norm(v["x"] - a["x"]) / np.linalg.norm(a["x"])
    dh = np.max(np.abs(v["hist"] - a["hist"]) / a["hist"])
    print(f"{k:12s} vs lag0: field {dx:.2e}, history {dh:.2e}, last presid {v['hist'][-1]:.3e}")
