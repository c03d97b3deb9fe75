#!/bin/bash
# Round-4 GPU session: selected GPU tests + config 5 profile (r4_check.sh), then the config-5
# MFMA A/B over lib/variants (mf_ab.sh), then the SQ counter passes (pmc_config5.sh).
# usage: tools/r4_session.sh TAG "TESTFILES" VARIANT...
TAG=$1; shift
TESTS=$1; shift
R=$GRAFT_REPO_ROOT
bash $R/tools/r4_check.sh $TAG $TESTS
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd $R
if [ $# -gt 0 ]; then bash tools/mf_ab.sh mfab_$TAG "$@" || exit $?; fi
bash tools/pmc_config5.sh $TAG || exit $?
exit $rc
