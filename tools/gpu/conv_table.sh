# Per-layer conv table (time + PMC HBM bytes):  gpurun -- bash tools/gpu/conv_table.sh TAG
set -o pipefail
T=${1:-r02}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python tools/conv_bench.py --iters 5 --json-out gpurun_out/ct_$T.json --sequence-out gpurun_out/cts_$T.json > gpurun_out/ct_$T.log 2>&1 || { echo "timing failed"; tail gpurun_out/ct_$T.log; exit 1; }
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/ctpmc_f_$T -o p -- python $R/tools/conv_bench.py --iters 2 --sequence-out $R/gpurun_out/ctsf_$T.json > $R/gpurun_out/ctpf_$T.log 2>&1 || { echo "pmc fetch failed"; tail $R/gpurun_out/ctpf_$T.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/ctpmc_w_$T -o p -- python $R/tools/conv_bench.py --iters 2 --sequence-out $R/gpurun_out/ctsw_$T.json > $R/gpurun_out/ctpw_$T.log 2>&1 || { echo "pmc write failed"; tail $R/gpurun_out/ctpw_$T.log; exit 1; }
cd $R
python tools/conv_layer_table.py gpurun_out/ct_$T.json gpurun_out/ctsf_$T.json gpurun_out/ctpmc_f_$T gpurun_out/ctpmc_w_$T gpurun_out/conv_layers_$T
