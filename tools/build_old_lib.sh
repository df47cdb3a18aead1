# build libllp_hip.so of a git revision (default HEAD) into tools/bin/old/ for same-box A/B (tools/gpu_lib_ab.sh)
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
rm -rf /tmp/llp_old && git worktree add -f /tmp/llp_old $REV > /dev/null 2>&1 || { git worktree prune; git worktree add -f /tmp/llp_old $REV > /dev/null; }
python /tmp/llp_old/linkless-link-prediction_amd/build_lib.py > /dev/null
mkdir -p tools/bin/old && cp /tmp/llp_old/linkless-link-prediction_amd/libllp_hip.so tools/bin/old/
git worktree remove --force /tmp/llp_old
echo "tools/bin/old/libllp_hip.so <- $(git rev-parse --short $REV)"
