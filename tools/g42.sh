# round-2 final refresh: full GPU suite, smoke, default bench line, 4K fp16 line + its kernel stats
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/g42
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
echo bench ok
timeout -k 10 300 python bench.py --precision fp16 --height 2160 --width 3840 --compare "" --host-pipeline 0 --no-cpu-baseline > $O/bench_4k_fp16.json 2> $O/bench_4k_fp16.err || exit $?
echo 4k ok
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof4k -o run --output-format csv -- python3 $R/bench.py --precision fp16 --height 2160 --width 3840 --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 > $R/$O/prof4k.log 2>&1 || exit $?
echo prof4k ok
