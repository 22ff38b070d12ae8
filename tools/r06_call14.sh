set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_recipes.sh trace ns || exit $?
bash tools/gpu_recipes.sh pmc ns || exit $?
bash tools/gpu_recipes.sh trace ns8 --blocks 8 --block-size 15625 --K 4 || exit $?
bash tools/gpu_recipes.sh stall ns || exit $?
bash tools/gpu_recipes.sh configs r06c || exit $?
