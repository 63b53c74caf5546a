cd $GRAFT_REPO_ROOT
for cfg in "VD_PLATE_S2D=1 VD_SSH_FUSE=1" "VD_PLATE_S2D=0 VD_SSH_FUSE=1" "VD_PLATE_S2D=1 VD_SSH_FUSE=0" "VD_PLATE_S2D=1 VD_SSH_FUSE=1"; do
  env $cfg timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err || exit 1
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json)"
done
