# Round-6 occupancy A/B of the b40 sibling kernel: each
# variant binary (scripts/ubench/sib_check.hip, XREF=1: the production kernel
# as reference in the same process) timed on the bench field, then its two
# counter passes (scripts/ubench/pmc_sib.sh).
set -e -o pipefail
B="scripts/ubench/sib_check_o_3_512_100 scripts/ubench/sib_check_o_3_1024_100 scripts/ubench/sib_check_o_2_768_1 scripts/ubench/sib_check_o_2_768_100 scripts/ubench/sib_check_o_2_512_100 scripts/ubench/sib_check_o_3_768_1"
bash scripts/ubench/run_checks.sh gpurun_out/occ_times.log "1916284264916 1000000000 5" $B
for b in $B; do bash scripts/ubench/pmc_sib.sh occ_${b##*_o_} $b; done
