#!/bin/bash
# Runs gpu.sh recipes in order (one argument per recipe line, e.g. "tests t1 tests/x.py").
# A failing recipe (test assertion, non-zero exit) does not stop the next one; a time limit,
# abort or segfault (124, 134, 137, 139) does - nothing more touches the GPU after it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
worst=0
for step in "$@"; do
    echo "=== $step"
    # shellcheck disable=SC2086
    bash tools/gpu.sh $step
    rc=$?
    echo "=== rc=$rc"
    case $rc in 124|134|137|139) exit $rc ;; esac
    [ $rc -ne 0 ] && worst=$rc
done
exit $worst
