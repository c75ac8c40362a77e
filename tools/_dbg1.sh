set -o pipefail
OUT=gpurun_out/dbg1
mkdir -p $OUT
ZKFL_LIB=build_ab/cur/libzkfl.so timeout -k 10 200 python -u -m pytest tests/test_cli.py -v --timeout 150 --timeout-method thread -m gpu > $OUT/cli_cur.log 2>&1; echo "cur rc=$?"; tail -n 2 $OUT/cli_cur.log
timeout -k 10 200 python -u -m pytest tests/test_cli.py -v --timeout 150 --timeout-method thread -m gpu > $OUT/cli_new.log 2>&1; echo "new rc=$?"; tail -n 2 $OUT/cli_new.log
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/all_new.log 2>&1; echo "all rc=$?"; grep -E "FAILED|ERROR|passed|failed" $OUT/all_new.log | tail -n 15
