set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_unet.py tests/test_gpu_b1024.py tests/test_gpu_schedule.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/oc2_pytest.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/oc2_pytest.log | tail -40; exit 1; }
tail -1 gpurun_out/oc2_pytest.log
timeout -k 10 120 python tools/conv_bench.py --layers out_conv1,out_conv2,enc1.conv2 --iters 20 > gpurun_out/oc2_conv.log 2>&1 || { echo "conv_bench failed"; tail -20 gpurun_out/oc2_conv.log; exit 1; }
cat gpurun_out/oc2_conv.log
for r in 1 2 3; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-live-traffic --steps 20 > gpurun_out/oc2_bench_$r.json 2> gpurun_out/oc2_bench_$r.err || { echo "bench failed"; tail gpurun_out/oc2_bench_$r.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/oc2_bench_$r.json')); print(d['ms_per_step'], d['value'], d['roofline']['forward']['train']['ms'], d['roofline']['forward']['eval']['ms'])"
done
