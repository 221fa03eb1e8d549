#!/bin/bash
# Several GPU check scripts in one box session; stops at a timeout / abort / segfault
# (exit 124, 134, 137, 139) so nothing else runs on a GPU that may be in trouble.
for step in "$@"; do
  echo "=== $step"
  bash -c "$step"
  rc=$?
  echo "=== rc $rc"
  case $rc in 124|134|137|139) echo "stopping after rc $rc"; exit $rc;; esac
done
