# Round-5 measurement on one GPU, in phases (one gpurun call each; every GPU
# step under its own time limit via scripts/gpu.sh or timeout, the script
# stops at the first failure):
#   bash scripts/r05_measure.sh bench    the default bench command under rocprofv3
#                                        (kernel trace + stats) and its --pmc passes
#                                        (one counter group per pass) -> scripts/pmc_bench.py
#   bash scripts/r05_measure.sh configs  every BASELINE config, the whole massive field
#                                        and its 8 dealt shares (floor 250 and 64)
#   bash scripts/r05_measure.sh bases    per-base PMC passes of the detailed kernel
#                                        (bench.py --base B --mode detailed, 1e9 at the
#                                        range start) -> scripts/pmc_bases.py
#   bash scripts/r05_measure.sh massive  PMC passes of the massive field's
#                                        msd_wave_kernel at floors 250 and 64
set -e -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
S="bash scripts/gpu.sh"
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"
case "$1" in
bench)
    $S prof default
    $S pmc busy "VALUBusy"
    $S pmc sq "$SQ"
    $S pmc fetch "FETCH_SIZE"
    $S pmc write "WRITE_SIZE" ;;
configs)
    timeout -k 10 500 python3 -u scripts/bench_configs.py --bases all > gpurun_out/configs.jsonl 2> gpurun_out/configs.err ;;
bases)
    for b in ${PMC_BASES:-40 52 53 54 64 65 80}; do
        $S pmc "b${b}_sq" "$SQ" --base "$b" --mode detailed --steps 3 --warmup 1
        $S pmc "b${b}_busy" "VALUBusy" --base "$b" --mode detailed --steps 3 --warmup 1
    done ;;
massive)
    cd /tmp && export TMPDIR=/tmp
    for fl in 250 64; do
        timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d "$R/gpurun_out/pmc_massive${fl}_sq" -o p -- \
            python3 "$R/scripts/massive_1gpu.py" 1 "$fl" > "$R/gpurun_out/pmc_massive${fl}_sq.log" 2>&1
        timeout -s KILL 120 rocprofv3 --pmc VALUBusy --output-format csv -d "$R/gpurun_out/pmc_massive${fl}_busy" -o p -- \
            python3 "$R/scripts/massive_1gpu.py" 1 "$fl" > "$R/gpurun_out/pmc_massive${fl}_busy.log" 2>&1
    done ;;
*)
    echo "usage: bash scripts/r05_measure.sh bench|configs|bases|massive" >&2
    exit 2 ;;
esac
