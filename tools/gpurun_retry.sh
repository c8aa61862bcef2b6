# Client-side wrapper: run one gpurun call; if the pool reports that no box
# was available or that it is backing off (nothing ran, nothing charged), wait
# as long as it asks (or 120 s) and submit the same call again, up to 8 times.
# A call that ran -- whatever its exit status -- is never resubmitted.
#   bash tools/gpurun_retry.sh <timeout-seconds> '<command>'
T=$1
CMD=$2
for attempt in 1 2 3 4 5 6 7 8; do
  out=$(timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" 2>&1)
  rc=$?
  echo "$out" | tail -4
  if ! echo "$out" | grep -q "status=transient\|no free box\|backing off\|slot(s) on this pod are busy"; then
    exit $rc
  fi
  wait_s=$(echo "$out" | grep -o "retry in [0-9]*s" | grep -o "[0-9]*" | tail -1)
  wait_s=$(( ${wait_s:-90} + 30 ))
  [ $wait_s -lt 120 ] && wait_s=120
  echo "[gpurun_retry] attempt $attempt: nothing ran; retrying in $wait_s s"
  sleep $wait_s
done
exit 3
