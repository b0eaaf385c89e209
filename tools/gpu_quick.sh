# Quick GPU check: GMRES / SpMV parity tests and bench lines at BASELINE configs 2 and 3.
# usage: tools/gpu_quick.sh TAG
set -u
TAG=${1:-q}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 100 > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['gmres'])" $OUT/bench_c$c.json
done
