# Round-5 measurement on one GPU (each step under its own limit via
# scripts/gpu.sh or timeout; stops at the first failure):
#  - the default bench command under rocprofv3 (kernel trace + stats) and its
#    --pmc passes (one counter group per pass) -> scripts/pmc_bench.py;
#  - per-base PMC passes of the detailed kernel (b40, b52-54, b64, b65, b80:
#    bench.py --base B --mode detailed, 1e9 at the range start) ->
#    scripts/pmc_bases.py;
#  - every BASELINE config, the whole massive field and its 8 dealt shares;
#  - PMC passes of the massive field's msd_wave_kernel.
set -e -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
S="bash scripts/gpu.sh"
$S prof default
$S pmc busy "VALUBusy"
$S pmc sq "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"
$S pmc fetch "FETCH_SIZE"
$S pmc write "WRITE_SIZE"
for b in ${PMC_BASES:-40 52 53 54 64 65 80}; do
    $S pmc "b${b}_sq" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE" \
        --base "$b" --mode detailed --steps 3 --warmup 1
    $S pmc "b${b}_busy" "VALUBusy" --base "$b" --mode detailed --steps 3 --warmup 1
done
timeout -k 10 300 python3 -u scripts/bench_configs.py --bases all > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES \
    GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_massive_sq" -o p -- \
    python3 "$R/scripts/massive_1gpu.py" 1 > "$R/gpurun_out/pmc_massive_sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc VALUBusy --output-format csv -d "$R/gpurun_out/pmc_massive_busy" -o p -- \
    python3 "$R/scripts/massive_1gpu.py" 1 > "$R/gpurun_out/pmc_massive_busy.log" 2>&1
