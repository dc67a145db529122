# persistent h4 (64-column tiles): equality tests, per-layer timing, forward, bench
#   gpurun -- bash tools/gpu/r04h.sh TAG
set -o pipefail
T=${1:-r04h}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_h4.py tests/test_gpu_unet.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_$T.log
[ $rc = 0 ] || { grep -E "Error|assert" gpurun_out/pytest_$T.log | head -20; exit $rc; }
timeout -k 10 150 python tools/conv_bench.py --layers enc1.conv2,dec1.conv1,dec1.conv2,enc2.conv1,enc2.conv2,bridge.3,dec3.conv1,dec2.conv1 --only fwd,dgrad --iters 10 > gpurun_out/layers_$T.txt 2>&1 || exit 1
cat gpurun_out/layers_$T.txt
for M in eval train; do
  timeout -k 10 120 python tools/fwd_bench.py --mode $M --iters 20 > gpurun_out/fwd_${T}_$M.json 2> gpurun_out/fwd_${T}_$M.err || exit 1
  cat gpurun_out/fwd_${T}_$M.json
done
timeout -k 10 300 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
cat gpurun_out/bench_$T.json | cut -c1-300
