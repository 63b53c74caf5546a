# round-2 profiles of the fp32 (fp16-pair) headline + the 4K fp16 line (BASELINE config 5, one GPU)
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/g21
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 > $R/$O/prof.log 2>&1 || exit $?
echo prof ok
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 > $R/$O/pmc_fetch.log 2>&1 || exit $?
echo fetch ok
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timing --compare "" --host-pipeline 0 > $R/$O/pmc_write.log 2>&1 || exit $?
echo write ok
cd $R
timeout -k 10 300 python bench.py --precision fp16 --height 2160 --width 3840 --compare "" --host-pipeline 0 --no-cpu-baseline > $O/bench_4k_fp16.json 2> $O/bench_4k_fp16.err || exit $?
echo 4k ok
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof4k -o run --output-format csv -- python3 $R/bench.py --precision fp16 --height 2160 --width 3840 --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 > $R/$O/prof4k.log 2>&1 || exit $?
echo prof4k ok
