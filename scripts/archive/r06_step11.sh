# round 6, after the closing run: the per-term breakdown of the final 8-wave program (set planes, R = 8, wave priority)
# and the object-API grid on this box
set -o pipefail
O=gpurun_out/r06_s11
mkdir -p $O
DIAGS="s8inline s8noread s8noown s8nobar s8nocombo" bash scripts/archive/r06_unit_breakdown.sh $O/unit > /dev/null || exit $?
grep -E "^==|enc_ms" $O/unit/sweep.txt | paste - - | sed 's/"variant": "bitsliced-jump-shared-8w", "tile_rows": 0, //' | cut -c1-200
timeout -k 10 600 build/object_api_bench > $O/object_api_grid.jsonl 2> $O/object_api_grid.err || { tail $O/object_api_grid.err; exit 1; }
echo "all done"
