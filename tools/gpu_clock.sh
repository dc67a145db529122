# effective shader clock during a kernel: GRBM_GUI_ACTIVE (GPU-busy cycles) / kernel duration,
# for the MFMA microbenchmark and for the h3 forward conv (bridge.3), normal and pure-MFMA (dbg 31)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $R/gpurun_out/clk_peak -o p -- $R/tools/mfma_peak > $R/gpurun_out/clk_peak.log 2>&1 || { echo "peak pass failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $R/gpurun_out/clk_conv -o p -- python $R/tools/conv_bench.py --layers bridge.3 --only fwd --iters 3 > $R/gpurun_out/clk_conv.log 2>&1 || { echo "conv pass failed"; exit 1; }
SRPDE_CONV_DBG=31 timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $R/gpurun_out/clk_conv31 -o p -- python $R/tools/conv_bench.py --layers bridge.3 --only fwd --iters 3 > $R/gpurun_out/clk_conv31.log 2>&1 || { echo "conv31 pass failed"; exit 1; }
cd $R
python tools/clock_summary.py gpurun_out/clk_peak mfma_
python tools/clock_summary.py gpurun_out/clk_conv conv_fwd_h3
python tools/clock_summary.py gpurun_out/clk_conv31 conv_fwd_h3
