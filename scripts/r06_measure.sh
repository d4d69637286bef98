# Round-6 measurement on one GPU, in phases (one gpurun call each; every GPU
# step under its own time limit via scripts/gpu.sh or timeout, the script
# stops at the first failure):
#   bash scripts/r06_measure.sh occupancy  b40 sibling-kernel occupancy A/B (VERDICT r05
#                                          item 1): A/B harness variants (build them with
#                                          scripts/ubench/sib_check.hip, see occupancy_ab.txt)
#                                          timed on the bench field, two counter passes each
#   bash scripts/r06_measure.sh small      small-field variants (item 5): GPU tests, then
#                                          the probe build's NICE_FD2_SMALLV kernels and
#                                          tagged vs untagged result words, and phase stamps
#   bash scripts/r06_measure.sh final      the final library: GPU tests, the default bench,
#                                          its rocprofv3 kernel trace + stats and --pmc
#                                          passes, every BASELINE config and per-base field
set -e -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
S="bash scripts/gpu.sh"
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"
case "$1" in
occupancy)
    B="scripts/ubench/sib_check_o_3_512_100 scripts/ubench/sib_check_o_3_1024_100 scripts/ubench/sib_check_o_2_768_1"
    B="$B scripts/ubench/sib_check_o_2_768_100 scripts/ubench/sib_check_o_2_512_100 scripts/ubench/sib_check_o_3_768_1"
    bash scripts/ubench/run_checks.sh gpurun_out/occ_times.log "1916284264916 1000000000 5" $B
    for b in $B; do bash scripts/ubench/pmc_sib.sh "occ_${b##*_o_}" "$b"; done ;;
small)
    $S tests
    export KNOB_ROUNDS=5
    timeout -k 10 200 python3 scripts/knob_sweep.py NICE_FD2_SMALLV 0,1,2,3 40:1e6 80:1e6 40:1e5 40:9e6 80:9e6 \
        40:1e6:0.5 80:1e6:0.5 > gpurun_out/small_v.log 2>&1
    timeout -k 10 200 python3 scripts/knob_sweep.py NICE_FD2_UNTAGGED ,1 40:1e6 80:1e6 40:1e5 > gpurun_out/small_tag.log 2>&1
    for v in 0 1 2 3; do
        NICE_FD2_SMALLV=$v timeout -k 10 120 python3 scripts/fd2_stamps.py 40:1e6 80:1e6 > gpurun_out/stamps_v$v.log 2>&1
    done ;;
final)
    $S tests
    $S bench final
    $S prof default
    $S pmc busy "VALUBusy"
    $S pmc sq "$SQ"
    $S pmc fetch "FETCH_SIZE"
    $S pmc write "WRITE_SIZE"
    timeout -k 10 500 python3 -u scripts/bench_configs.py --bases all > gpurun_out/configs.jsonl 2> gpurun_out/configs.err ;;
*)
    echo "usage: bash scripts/r06_measure.sh occupancy|small|final" >&2
    exit 2 ;;
esac
