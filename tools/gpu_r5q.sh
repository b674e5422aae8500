# round 5 (q): byte-map PACK variants on one box, interleaved, with the floors
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
T="struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed ref_struct ref_strange"
for rep in 1 2; do
for v in "MX_CONV_BMAP_SPAN=24576 MX_CONV_BMAP_UNROLL=0" "MX_CONV_BMAP_SPAN=24576" "MX_CONV_BMAP_SPAN=49152 MX_CONV_BMAP_UNROLL=0" "MX_CONV_BMAP_SPAN=49152" "MX_CONV_BMAP_DW=0" "MX_CONV_BMAP_SPAN=12288"; do
  echo "== $v (rep $rep)" >> $O/conv_ab_r5q.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack $T >> $O/conv_ab_r5q.txt 2>&1 || exit $?
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack $T >> $O/conv_ab_r5q.txt 2>&1 || exit $?
done
timeout -k 10 120 ./tools/pack_floor_probe $(python tools/pack_floor_args.py $((256<<20))) >> $O/pack_floor_r5q.txt 2>&1 || exit $?
timeout -k 10 120 ./tools/pack_floor_probe $(python tools/pack_floor_args.py $((1<<30))) >> $O/pack_floor_r5q.txt 2>&1 || exit $?
done
grep -v amdgpu.ids $O/conv_ab_r5q.txt | grep -v "^$"
grep -E "struct_char|indexed_f32|blacs|ref_struct|ref_strange" $O/pack_floor_r5q.txt
