# Client-side wrapper: run one gpurun call; if the pool reports that no box
# was available or the box was lost before the command started (nothing ran,
# nothing charged), wait and submit the same call again, up to 6 times.  A
# call that ran -- whatever its exit status -- is never resubmitted.
#   bash tools/gpurun_retry.sh <timeout-seconds> '<command>'
T=$1
CMD=$2
for attempt in 1 2 3 4 5 6; do
  out=$(timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" 2>&1)
  rc=$?
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=ok\|status=fail\|status=timeout\|rc=[0-9]"; then
    if ! echo "$out" | grep -q "status=transient"; then
      exit $rc
    fi
  fi
  if [ $rc -ne 3 ] && ! echo "$out" | grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|stopped responding while being prepared\|taken away by the GPU service\|backing off"; then
    exit $rc
  fi
  echo "[gpurun_retry] attempt $attempt: nothing ran; retrying in 90 s"
  sleep 90
done
exit 3
