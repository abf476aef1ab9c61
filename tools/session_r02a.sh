cd "${GRAFT_REPO_ROOT}"
bash tools/session_r02.sh test || exit $?
bash tools/sweep.sh "" "--tile-order 0" "" "--tile-order 0" "--tail-split 0" "--tile-order 0 --tail-split 0" "" || exit $?
bash tools/session_r02.sh prof || exit $?
