# round 6: four ranks on the lease's one GPU (device = LOCAL_RANK mod device count): the default weak-scaling workload
# and configs[4]'s whole job split four ways -- the N = 4 code path (rank contexts, gloo gathers, the split) on hardware
set -o pipefail
O=gpurun_out/r06_n4
mkdir -p $O
timeout -k 10 400 python bench.py --gpus 4 --no-cpu-baseline --no-ceiling > $O/default_n4_onegpu.json 2> $O/default_n4_onegpu.err || { tail -20 $O/default_n4_onegpu.err; exit 1; }
grep '^{' $O/default_n4_onegpu.json | cut -c1-400
timeout -k 10 600 python bench.py --gpus 4 --workload config5 --no-cpu-baseline --no-ceiling > $O/config5_n4_onegpu.json 2> $O/config5_n4_onegpu.err || { tail -20 $O/config5_n4_onegpu.err; exit 1; }
grep '^{' $O/config5_n4_onegpu.json | cut -c1-400
echo "all done"
