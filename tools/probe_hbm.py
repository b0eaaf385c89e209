"""Streaming roofline probes for the stencil's byte mix (see csrc/probe.hip).
usage: python tools/probe_hbm.py [n] [rotating pairs, default 3; 1 = same buffers]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402
from helmholtz_preconditioner_amd import _ffi  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
om, h, eta = H.problem_params(n, 12, 100.0, 2.0)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, H.marmousi_like_c_mat(n))
R = int(sys.argv[2]) if len(sys.argv) > 2 else 3  # rotating (x, y) pairs: cold inputs
xs, ys = [A.vector() for _ in range(R)], [A.vector() for _ in range(R)]
for k, v in enumerate(xs):
    v.fill_hash(1 + k)
raw = lambda v: v.handle.value if isinstance(v.handle, ctypes.c_void_p) else v.handle
hx = (ctypes.c_void_p * R)(*[raw(v) for v in xs])
hy = (ctypes.c_void_p * R)(*[raw(v) for v in ys])
print(f"n={n}, {R} rotating (x, y) pairs")
names = ["1pt/lane u16 ic8 y16", "2pt/lane adjacent (ic16, u/y 32B stride)",
         "2pt/lane wave-strided (ic8)", "copy y=u", "read-only u+ic", "1pt/lane nontemporal",
         "copy 2pt/lane adjacent", "stencil traversal, XCD map (no arithmetic)",
         "stencil traversal, blockIdx order", "stencil traversal, 8-row bands",
         "stencil traversal, 16-row bands", "stencil traversal, 64-row bands",
         "stencil traversal, 128-row bands", "naive 5-point gather, blockIdx order",
         "naive 5-point gather, XCD row ranges", "copy, NT loads + NT stores",
         "copy, cached loads + NT stores", "tile shape R6: own rows only",
         "tile shape R6: + halo rows", "tile shape R6: + halo + edge loads",
         "tile shape R6: + halo + edge + tables", "tile shape R12: own rows only"]
kinds = [int(k) for k in os.environ.get("PROBE_KINDS", ",".join(map(str, range(22)))).split(",")]
km, bpp = ctypes.c_double(), ctypes.c_int()
for blocks in (2048, 8192, 32768):
    for kind in kinds:
        if (7 <= kind <= 14 or kind >= 17) and blocks != 2048:
            continue  # the marching probes size their own grid
        best = 1e9
        for _ in range(3):
            _ffi.check(_ffi.lib.hh_op_probe_stream_set(A.handle, kind, blocks, hx, hy, R, 21,
                                                       ctypes.byref(km), ctypes.byref(bpp)))
            best = min(best, km.value)
        print(f"blocks {blocks:6d} kind {kind} {names[kind]:42s} {best*1e3:8.1f} us "
              f"{bpp.value*n*n/(best*1e-3)/1e9:7.0f} GB/s", flush=True)
