#!/bin/bash
# r05c (L1-3 sorted runs) then r05b (sorted-run k_match2 A/B); r05b runs only
# if r05c ended normally (0) or on a plain test failure (1)
./tools/jobs/r05c.sh
rc=$?
echo "r05c rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
./tools/jobs/r05b.sh
