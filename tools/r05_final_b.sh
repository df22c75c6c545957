#!/bin/bash
# round-5 closing pass, second box: cfg4 / cfg5 / yadif / cfg2 from nv12 (line, trace, PMC) + the e2e lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SKIP_TESTS=1 bash tools/r05_final.sh ${1:-r05f} cfg4 cfg5 yadif cfg2nv12
