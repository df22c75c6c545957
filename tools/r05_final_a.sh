#!/bin/bash
# round-5 closing pass, first box: the GPU suite + smoke, then cfg2 / cfg1 / cfg3 (line, trace, PMC)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SKIP_E2E=1 bash tools/r05_final.sh ${1:-r05f} cfg2 cfg1 cfg3
