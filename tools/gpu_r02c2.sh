#!/bin/bash
# config 2 (1024^2 Jacobi GMRES): fused last-block Krylov kernels on / off (HH_KRYLOV_FUSE), then the
# GMRES parity tests with the default (on)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r02c2}
mkdir -p "$OUT"
for rev in 2 0 1 3 2 0; do  # (HH_KRYLOV_FUSE bits)
  HH_KRYLOV_FUSE=$rev timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline > "$OUT/c2_rev$rev.log" 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/c2_rev$rev.log') if l.startswith('{')][-1]); print('rev $rev', d['gmres'])"
done
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gmres.py tests/test_gpu_configs.py tests/test_gpu_krylov_modes.py tests/test_gpu_variants.py tests/test_gpu_errors.py tests/test_gpu_sweep.py > "$OUT/t_gmres.log" 2>&1; rc=$?
tail -3 "$OUT/t_gmres.log"; exit $rc
