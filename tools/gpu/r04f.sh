# h4 with 64-column tiles / W = 40: equality tests, per-layer timing h4 vs h3r, the forward and the bench
#   gpurun -- bash tools/gpu/r04f.sh TAG
set -o pipefail
T=${1:-r04f}
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_h4.py tests/test_gpu_kernels.py tests/test_gpu_unet.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_$T.log
[ $rc = 0 ] || exit $rc
L=enc1.conv2,dec1.conv1,dec1.conv2,enc2.conv1
SRPDE_H4=0 timeout -k 10 120 python tools/conv_bench.py --layers $L --only fwd,dgrad --iters 10 > gpurun_out/w40_h3r_$T.txt 2>&1 || exit 1
timeout -k 10 120 python tools/conv_bench.py --layers $L --only fwd,dgrad --iters 10 > gpurun_out/w40_h4_$T.txt 2>&1 || exit 1
cat gpurun_out/w40_h3r_$T.txt gpurun_out/w40_h4_$T.txt
timeout -k 10 300 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
cat gpurun_out/bench_$T.json
