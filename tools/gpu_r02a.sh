set -e
O=gpurun_out/r02a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --tb=short --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
