set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
RSLRL_AMD_LIB=rsl_rl_amd/lib/variants/gaestamps/librslrl_amd.so timeout -k 10 120 python3 scripts/gae_stamps.py > gpurun_out/r6/gae_stamps.log 2>&1
echo rc=$?
tail -5 gpurun_out/r6/gae_stamps.log | cut -c1-1500
