set -o pipefail
# the committed build as the driver runs it: smoke, then the GPU suite
out=gpurun_out/r6last; mkdir -p $out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; echo "suite rc=$?"; tail -3 $out/tests.log
