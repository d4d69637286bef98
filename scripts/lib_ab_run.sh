# Same-box A/B of two library builds (scripts/lib_ab.py): an earlier build
# copied into ab_old/ (package + libnice_hip.so) against the tree's, each in
# its own process, interleaved, two passes.  Remove ./ab_old from
# .gpurunignore for the run (it is listed there so ordinary calls skip it).
#   gpurun -- bash scripts/lib_ab_run.sh "80:1e9 60:1e9 40:1e6" [log]
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
log=${2:-gpurun_out/lib_ab.log}
for i in 1 2; do
  for d in ab_old .; do
    timeout -k 10 120 python3 scripts/lib_ab.py $d $1 >> $log 2>&1
  done
done
