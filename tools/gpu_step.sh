# sourced by the tools/gpu_r03*.sh scripts: run one GPU step under a time
# limit; a test failure (rc 1-2) is recorded and the script goes on, a
# fault, abort, kill or time limit (any other nonzero rc) ends it
step() {
  local name=$1; shift
  "$@"
  local rc=$?
  echo "step $name rc=$rc" >> $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ]; then exit $rc; fi
  return 0
}
