# Round-3 measurement of the default bench command: the bench line, its
# rocprofv3 kernel trace, and rocprofv3 --pmc passes of the SAME command (one
# counter group per pass) for roofline.frac_hw / traffic.
set -e -o pipefail
S="bash scripts/gpu.sh"
$S bench default
$S prof default
$S pmc busy "VALUBusy"
$S pmc sq "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"
$S pmc fetch "FETCH_SIZE"
$S pmc write "WRITE_SIZE"
