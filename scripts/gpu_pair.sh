#!/bin/bash
# Run two GPU scripts in one gpurun call: the second only if the first ended normally (exit 0 or
# an ordinary failure such as a failed test) -- never after a time limit, abort or fault.
A=$1; B=$2
bash $A; rc=$?
echo "== $A rc=$rc"
case $rc in 124|134|137|139) exit $rc ;; esac
bash $B; rc2=$?
echo "== $B rc=$rc2"
[ $rc -ne 0 ] && exit $rc
exit $rc2
