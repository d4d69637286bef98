# Run A/B check binaries one after another on the GPU box; a binary exits 0
# (match) or 1 (mismatch); any other status (fault, abort, timeout) stops the
# run there.  Usage: bash scripts/ubench/run_checks.sh OUT "ARGS" BIN...
out=$1; args=$2; shift 2
: > "$out"
for b in "$@"; do
    timeout -k 5 90 "$b" $args >> "$out" 2>&1
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$b: exit $rc, stopping" >> "$out"; exit $rc; fi
done
exit 0
