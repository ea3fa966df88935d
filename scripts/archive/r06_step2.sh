# round 6, second GPU call: the per-term breakdown of the 8-wave encode unit (diagnostic builds, interleaved), then
# the PMC traffic passes of the shipped bench at head (encode product and decode product)
set -o pipefail
O=gpurun_out/r06_s2
mkdir -p $O
bash scripts/archive/r06_unit_breakdown.sh $O/unit > /dev/null || exit $?
grep -E "^==|enc_ms" $O/unit/sweep.txt | paste - - | cut -c1-200
bash scripts/pmc_bench.sh || exit $?
cp -r gpurun_out/pmc_bench $O/pmc_bench
echo "all done"
