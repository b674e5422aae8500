# convertor A/B: pipelined pack geometry, and the 32-byte write sector of gapped unpack
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T="struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed ref_lower_matrix_47"
for g in 0 1 2 3; do
  echo "GEOM=$g" | tee -a $O/r2d_geom.txt
  MX_CONV_PIPE_GEOM=$g timeout -k 10 120 python -u tools/conv_probe.py --dirs pack $T >> $O/r2d_geom.txt 2>&1 || exit 1
done
cat $O/r2d_geom.txt
V="vec:f32:1:2 vec:f32:4:8 vec:f32:8:16 vec:f32:16:32 vec:f32:8:12 struct_char_d3_int_resized48"
timeout -k 10 120 python -u tools/conv_probe.py --dirs unpack $V > $O/r2d_unpack.txt 2>&1 || exit 1
cat $O/r2d_unpack.txt
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/r2d_pmc_$c -o run -- python3 tools/conv_probe.py --reps 1 --dirs unpack $V > $O/r2d_pmc_$c.log 2>&1 || exit 1
done
for g in 0 1; do
  MX_CONV_PIPE_GEOM=$g timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d $O/r2d_sq$g -o run -- python3 tools/conv_probe.py --reps 1 --dirs pack struct_char_d3_int_resized48 > $O/r2d_sq$g.log 2>&1 || exit 1
done
echo ok
