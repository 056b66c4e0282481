cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/f2
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/f2/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/f2/pytest.log | head; exit 1; }
tail -1 gpurun_out/f2/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/f2/bench.json 2> gpurun_out/f2/bench.err || { echo bench failed; exit 1; }
tail -1 gpurun_out/f2/bench.json | cut -c1-200
