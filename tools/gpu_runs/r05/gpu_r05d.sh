# r05d: the glue from 1, 2, 4 host threads on one GPU (tools/probes/mt_glue,
# VERDICT r04 weak #2), then the same under rocprofv3's HIP API trace
set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
export TMPDIR=/tmp
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $O/nproc.txt 2>/dev/null; taskset -p $$ >> $O/nproc.txt
timeout -k 10 300 tools/probes/mt_glue > $O/mt.json 2> $O/mt.err || exit 3
echo "mt ok" >> $O/steps.txt
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/prof -o mt -- tools/probes/mt_glue 4194304 CheckIPHeader > $O/mt_prof.json 2> $O/mt_prof.err || exit 4
echo "prof ok" >> $O/steps.txt
