cd "${GRAFT_REPO_ROOT}"
for c in C2 C3 C4; do CFG=$c timeout -k 10 600 bash tools/strip_probe.sh || exit $?; done
