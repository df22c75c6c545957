#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/r04_yadif.sh r04a || exit $?
bash tools/r04_hdr_ab.sh
bash tools/r04_l7ab.sh
