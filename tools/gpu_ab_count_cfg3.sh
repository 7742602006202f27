set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "^sweep|passed|failed|Error" "$OUT/$name.log" | tail -n 20; return $rc; }
step pytest_q 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "65 or stream_head or count or generated or fuzzed" || exit $?
step sweep3 400 python bench.py --sweep cfg3 --sweep-counts --steps 10 --warmup 3 --sweep-variants "8,2,2,0;0,0,0,65;0,0,0,64;8,2,2,0;0,0,0,65" || exit $?
step sweep4 400 python bench.py --sweep cfg4,cfg5 --steps 10 --warmup 3 --sweep-variants "0,0,0,64;0,0,0,38" || exit $?
step sweep4c 400 python bench.py --sweep cfg4,cfg5 --sweep-counts --steps 10 --warmup 3 --sweep-variants "0,0,0,64;0,0,0,38" || exit $?
echo ALLDONE
