set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_recipes.sh trace ns || exit $?
bash tools/gpu_recipes.sh pmc ns || exit $?
bash tools/gpu_recipes.sh configs r06 || exit $?
