# step NAME CMD... : run one GPU step; stop the whole call after a timeout, abort or crash.
step() {
    local name=$1; shift
    "$@"
    local rc=$?
    echo "[$name] rc=$rc"
    if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
        echo "[$name] fatal (timeout/abort/crash): stopping"
        exit $rc
    fi
    return 0
}
