# round-2 closing (256-channel streaming slices): full GPU suite, smoke, default bench line, kernel-trace + PMC profiles (fp32 headline)
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/g53
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
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 > $R/$O/prof.log 2>&1 || exit $?
echo prof ok
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 > $R/$O/pmc_fetch.log 2>&1 || exit $?
echo fetch ok
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 > $R/$O/pmc_write.log 2>&1 || exit $?
echo write ok
