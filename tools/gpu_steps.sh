#!/bin/bash
# Run GPU steps in order, each under its own time limit; an ordinary failure (exit 1, e.g. a red test)
# moves on, a fatal one (time limit 124/137, abort 134, segfault 139, signal) ends the call.
#   tools/gpu_steps.sh OUTDIR "name|seconds|command" ...
out=$1
shift
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc $(( $(date +%s) - start )) s"
  tail -n 4 "$out/$name.log"
  case $rc in
    0|1|2) ;;
    *) echo "== fatal exit $rc in $name: stopping"; exit $rc ;;
  esac
done
