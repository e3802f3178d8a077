set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/r6o; mkdir -p $O
T=rten-fork_amd/tools/stem_bench.py
for r in 1 2; do
echo -n "forced-stem " >> $O/stem.txt
RTENHIP_PW_VALU=800 timeout -k 10 120 python -u $T mobilenet_v2 128 50 2>/dev/null >> $O/stem.txt || exit 1
echo -n "tuned-no-stem " >> $O/stem.txt
RTENHIP_STEM=0 timeout -k 10 120 python -u $T mobilenet_v2 128 50 2>/dev/null >> $O/stem.txt || exit 1
done
cat $O/stem.txt
cd /tmp
RTENHIP_PW_VALU=800 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OLDPWD/$O/pmc -o run -- python3 $OLDPWD/$T mobilenet_v2 128 5 > $OLDPWD/$O/pmc.log 2>&1 || { tail -5 $OLDPWD/$O/pmc.log; exit 1; }
cd $OLDPWD
python3 rten-fork_amd/tools/pmc_kernels.py $O/pmc stem
rm -rf $O/pmc
