#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/r04_tm.sh || exit $?
bash tools/r04_co.sh
