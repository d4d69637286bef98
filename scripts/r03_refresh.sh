# Round-3 refresh on one GPU: the gpu tests, the default bench command under
# rocprofv3 (kernel trace + stats) and its --pmc passes (one counter group per
# pass), every BASELINE config and every FD base at 1e9, and the small-field
# phase stamps.  Each step under its own limit (scripts/gpu.sh); stops at the
# first failure.
set -e -o pipefail
S="bash scripts/gpu.sh"
$S tests
$S prof default
$S pmc busy "VALUBusy"
$S pmc sq "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"
$S pmc fetch "FETCH_SIZE"
$S pmc write "WRITE_SIZE"
timeout -k 10 300 python3 -u scripts/bench_configs.py --bases all > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
