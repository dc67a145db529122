# switch test with the term-level spatial-bias check, the attention-bias seed table, the cascade
# test, h4 timing after the barrier-count fix, and the bench
#   gpurun -- bash tools/gpu/r04e.sh TAG
set -o pipefail
T=${1:-r04e}
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_cascade.py tests/test_gpu_h4.py -q --timeout 240 \
  --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$T.log
[ $rc = 0 ] || [ $rc = 1 ] || exit $rc
timeout -k 10 200 python -u tools/diag_att_bias.py 10 > gpurun_out/attb_$T.txt 2>&1 || exit 1
cat gpurun_out/attb_$T.txt
timeout -k 10 120 python tools/conv_bench.py --layers bridge.3,dec3.conv1,dec2.conv1,enc2.conv2 --only fwd,dgrad \
  --iters 10 > gpurun_out/h4t_$T.txt 2>&1 || exit 1
cat gpurun_out/h4t_$T.txt
timeout -k 10 300 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
cat gpurun_out/bench_$T.json
exit $rc
