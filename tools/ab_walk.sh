L=volsync_amd/lib/var
LIBS=base=$L/w512base/libvsgpu.so,f8r8=$L/w256f8r8/libvsgpu.so,f16r8=$L/w256f16r8/libvsgpu.so,f8r12=$L/w256f8r12/libvsgpu.so
GPU_STEP_TIMEOUT=700 bash tools/gpu.sh py tools/ab.py --rounds 2 --timeout 300 --libs $LIBS -- bench.py --mode rsync --share 3/8 --per-gpu-gib 32 --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline && mv gpurun_out/py_ab.log gpurun_out/ab_share.log &&
GPU_STEP_TIMEOUT=700 bash tools/gpu.sh py tools/ab.py --rounds 2 --timeout 300 --libs $LIBS -- bench.py --mode rsync --steps 3 --warmup 1 --no-file-sum --no-cpu-baseline && mv gpurun_out/py_ab.log gpurun_out/ab_c4.log
