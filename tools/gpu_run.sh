#!/bin/bash
# One gpurun session: GPU tests, smoke, bench, optional rocprof. Each GPU step
# has its own time limit; a crash/abort/timeout (anything but exit 0/1) stops
# the script before the next GPU step.
#   bash tools/gpu_run.sh [tests|smoke|bench|prof|profp|pmc ...]   (profp: plate net alone)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=("$@")
[ ${#STEPS[@]} -eq 0 ] && STEPS=(tests smoke bench)
BENCH_ARGS=${BENCH_ARGS:-"--steps 20 --warmup 3"}
PROF_ARGS=${PROF_ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline"}
PMC_ARGS=${PMC_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline --no-timing"}
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu -x -q"}
PYTEST_K=${PYTEST_K:-}   # optional -k expression (may contain spaces)

run() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name: $*" | tee -a gpurun_out/steps.log
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
    tail -n 5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "== stopping after $name (rc=$rc)"; exit $rc
    fi
    return 0
}

for s in "${STEPS[@]}"; do
    case $s in
        tests) if [ -n "$PYTEST_K" ]; then run pytest_gpu 700 python -m pytest $PYTEST_ARGS -k "$PYTEST_K"
               else run pytest_gpu 700 python -m pytest $PYTEST_ARGS; fi ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 400 python bench.py $BENCH_ARGS ;;
        prof)  run prof${PROF_TAG:-} 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof${PROF_TAG:-} -o run --output-format csv -- python3 bench.py $PROF_ARGS ;;
        profp) run profp 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profp -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --faces 0 --plates 1 ;;
        pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py $PMC_ARGS &&
               run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py $PMC_ARGS ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
