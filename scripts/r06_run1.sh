set -e -o pipefail
bash scripts/gpu.sh tests
bash scripts/gpu.sh bench r06start
bash scripts/ubench/run_checks.sh gpurun_out/sib_repro.log "1916284264916 100000000 1" scripts/ubench/sib_check_q_2_768_2050 scripts/ubench/sib_check_q_2_768_2049 scripts/ubench/sib_check_q_2_512_2050 scripts/ubench/sib_check_q_3_768_4097
