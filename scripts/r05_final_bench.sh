#!/usr/bin/env bash
# Round-5 final bench lines (C2-C5 with CPU baselines, scripts/session.sh bench) and the C3 kernel
# levels (scripts/r05_s12.sh: literal, edited scene, uploaded geometry, const, generic, reference leaks).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PARTS="bench" TAG=r05 bash scripts/session.sh || exit $?
bash scripts/r05_s12.sh
