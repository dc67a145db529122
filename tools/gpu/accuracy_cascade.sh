# Config #5 on the current tree (verdict r4 #8): device data-gen + training with the reference config, the
# reference's resolution comparison (MAE / RMSE 80..640 against bilinear / bicubic), then the cascade bench
# line (latency + rmse_vs_gt640) on the trained checkpoint.   gpurun -- bash tools/gpu/accuracy_cascade.sh TAG
set -o pipefail
T=${1:-acc}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/e2e_accuracy.py --save gpurun_out/e2e_$T > gpurun_out/e2e_$T.json 2> gpurun_out/e2e_$T.err || { tail -20 gpurun_out/e2e_$T.err; exit 1; }
python -c "
import json; t=open('gpurun_out/e2e_$T.json').read(); d=json.loads(t[t.rfind(chr(10) + '{') + 1:])   # the summary follows the training log
print('epochs', d['epochs_run'], 'best', d['best_epoch'], 'val', d['best_val_loss'], 'wall', d['wall_s_generate_and_train'])
for r, t in d['resolution_comparison_mean_over_seeds'].items():
    print(r, {m: (round(v['mae_mean'] * 1e6, 2), round(v['rmse_mean'] * 1e6, 2)) for m, v in t.items() if isinstance(v, dict)})
"
timeout -k 10 400 python bench.py --workload cascade --checkpoint gpurun_out/e2e_$T/e2e_best_weights.pt --steps 10 --warmup 2 > gpurun_out/cascade_$T.json 2> gpurun_out/cascade_$T.err || { tail -10 gpurun_out/cascade_$T.err; exit 1; }
cat gpurun_out/cascade_$T.json
