set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 180 python -u rten-fork_amd/tools/fork_probe.py 2>&1 | grep -v amdgpu.ids
