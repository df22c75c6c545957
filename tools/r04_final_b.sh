#!/bin/bash
# round-4 closing pass, second box: cfg4 / cfg5 / yadif / cfg2 from nv12 (line, trace, PMC) + e2e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SKIP_TESTS=1 bash tools/r04_final.sh ${1:-r04f} cfg4 cfg5 yadif cfg2nv12
