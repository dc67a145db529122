set -o pipefail
cd $GRAFT_REPO_ROOT
for hp in 4 1 1000; do
  echo "== HP=$hp"; SRPDE_CONV_HP=$hp timeout -k 10 200 python tools/conv_bench.py --only fwd || exit 1
done
echo "== dgrad/wgrad (HP=4)"; timeout -k 10 200 python tools/conv_bench.py --only dgrad,wgrad
