set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decomp.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
BZG_DEC_DEBUG=1 timeout -k 10 300 python tools/prof_config.py text 2 decode > $O/dec.log 2>&1 || { echo "dec failed"; tail -20 $O/dec.log; exit 1; }
cat $O/dec.log
