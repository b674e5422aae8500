set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
# SQ counters of the tile convertor on the struct type (byte-granular pieces), one pass
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O/r1ak_sq -o run -- python3 tools/pmc_unpack.py struct_char_d3_int_resized48 2 > $O/r1ak_sq.txt 2>&1 || { tail -20 $O/r1ak_sq.txt; exit 1; }
tail -2 $O/r1ak_sq.txt
