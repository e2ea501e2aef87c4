#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/r3_ab.sh && TAG=r3p bash scripts/r3_profile.sh && TAG=r3k bash scripts/r3_cli.sh
