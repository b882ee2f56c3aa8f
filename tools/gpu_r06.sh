# Round-6 GPU steps (run on the GPU box from the repository root):  bash tools/gpu_r06.sh <step> [tag]
#   scl    SCL parity tests, then the same-process SCL variant A/B on the bench's AWGN input
#   tests  the whole -m gpu suite
#   bench  bench.py (default N=1 line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out
mkdir -p $O
step=$1
tag=${2:-r06}
case $step in
scl)
    timeout -k 10 400 python -u -m pytest tests/test_scl_gpu.py tests/test_mysn_gpu.py -x -q -rf --timeout 200 \
        --timeout-method thread > $O/${tag}_pytest_scl.log 2>&1 || { tail -30 $O/${tag}_pytest_scl.log; exit 1; }
    tail -2 $O/${tag}_pytest_scl.log
    SCL_INPUT=awgn SCL_ROUNDS=${ROUNDS:-3} timeout -k 10 300 python -u tools/scl_variants.py time \
        > $O/${tag}_scl_ab.txt 2>&1 || { cat $O/${tag}_scl_ab.txt; exit 1; }
    cat $O/${tag}_scl_ab.txt
    if [ -n "$MYSN" ]; then  # my_sn SCL_Dec default: exact f + fast-SCL
        SCL_INPUT=awgn SCL_FMODE=1 SCL_FLAGS=4 SCL_ROUNDS=2 timeout -k 10 300 python -u tools/scl_variants.py time \
            > $O/${tag}_scl_ab_mysn.txt 2>&1 || { cat $O/${tag}_scl_ab_mysn.txt; exit 1; }
        cat $O/${tag}_scl_ab_mysn.txt
    fi
    ;;
tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread \
        > $O/${tag}_pytest_gpu.log 2>&1 || { tail -40 $O/${tag}_pytest_gpu.log; exit 1; }
    tail -3 $O/${tag}_pytest_gpu.log
    ;;
bench)
    timeout -k 10 600 python -u bench.py > $O/${tag}_bench.json 2> $O/${tag}_bench.err || { tail -30 $O/${tag}_bench.err; exit 1; }
    cat $O/${tag}_bench.json
    ;;
*)
    echo "unknown step $step"; exit 2 ;;
esac
