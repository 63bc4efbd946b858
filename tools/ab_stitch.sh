# stitch merge A/B (round 3): the walk tests on the new library, then the
# share and C4-shape lines against the previous build
L=volsync_amd/lib/var
bash tools/gpu.sh tests tests/test_gpu_rsync.py -x && mv gpurun_out/gputests.log gpurun_out/gputests_rsync.log &&
GPU_STEP_TIMEOUT=700 bash tools/gpu.sh py tools/ab.py --rounds 2 --timeout 300 --libs base=$L/w512base/libvsgpu.so,new= -- bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline && mv gpurun_out/py_ab.log gpurun_out/ab_stitch_share.log &&
GPU_STEP_TIMEOUT=700 bash tools/gpu.sh py tools/ab.py --rounds 2 --timeout 300 --libs base=$L/w512base/libvsgpu.so,new= -- bench.py --mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline && mv gpurun_out/py_ab.log gpurun_out/ab_stitch_c4.log
