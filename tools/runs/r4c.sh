mkdir -p gpurun_out/r4c && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_gpu_configs.py -k "pipeline or batch_process or c2_bf16_720p_heads" -p no:cacheprovider > gpurun_out/r4c/tests.log 2>&1; tail -3 gpurun_out/r4c/tests.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline > gpurun_out/r4c/bench.json 2> gpurun_out/r4c/bench.err || exit 1
for c in 4 8 16 32; do timeout -k 10 200 python bench.py --steps 10 --warmup 3 --compare "" --no-cpu-baseline --host-pipeline 0 --option mosaic_cells=$c > gpurun_out/r4c/cells$c.json 2>> gpurun_out/r4c/bench.err || exit 1; done
