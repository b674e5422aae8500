# byte-map pack vs piece pack on the small dense types
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T="struct_char_d3_int_resized48 ref_struct ref_struct_char_double ref_strange indexed_f32_random ref_blacs_indexed ref_lower_matrix_47 ref_twice_two_doubles ref_struct_constant_gap_resized"
for b in 1 0; do
  echo "BMAP_PACK=$b" >> $O/r2s_ab.txt
  MX_CONV_BMAP_PACK=$b timeout -k 10 240 python -u tools/conv_probe.py --dirs pack $T >> $O/r2s_ab.txt 2>&1 || exit 1
done
grep -v amdgpu $O/r2s_ab.txt
echo ok
