#!/bin/bash
# Resident kernel cost split (profiling-only variants): default, no hand-offs, no rows, no barriers
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
W16=$PWD/tools/ubench/bin/w16/libpanofuse.so
VARIANTS="dbg1:PF_NOSIDE=1,PF_JRES_DBG=1 dbg5:PF_NOSIDE=1,PF_JRES_DBG=5 dbg9:PF_NOSIDE=1,PF_JRES_DBG=9 w16:PF_NOSIDE=1,PANOFUSE_LIB=$W16 w16dbg1:PF_NOSIDE=1,PF_JRES_DBG=1,PANOFUSE_LIB=$W16 w16dbg5:PF_NOSIDE=1,PF_JRES_DBG=5,PANOFUSE_LIB=$W16 w16dbg9:PF_NOSIDE=1,PF_JRES_DBG=9,PANOFUSE_LIB=$W16" TAG=_split bash tools/jres_probe.sh
