#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
for V in "" "TBLS_KEYS_COOP=0" "TBLS_SIG_COOP=0" "TBLS_KEYS_COOP=0 TBLS_SIG_COOP=0"; do
echo "== $V"; env $V timeout -k 10 120 python tools/dbg/kcoop_ab.py || exit $?
done
