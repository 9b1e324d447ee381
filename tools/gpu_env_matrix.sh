# The GPU suite under non-default runtime settings (every form must give the same bits):
# all-NT streaming, in-launch tickets everywhere, xGMI host mirror, no deferral / no coop.
set -o pipefail
mkdir -p gpurun_out/envm
i=0
for E in "LBFGS_NT=1" "LBFGS_TICKET=1" "LBFGS_XGMI_MIRROR=1 LBFGS_NT=0" "LBFGS_DEFER=0 LBFGS_COOP=0 LBFGS_REV=0"; do
  i=$((i+1))
  env $E timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/envm/pytest_$i.log 2>&1; rc=$?
  echo "[$E] rc=$rc $(tail -1 gpurun_out/envm/pytest_$i.log)"
  [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/envm/pytest_$i.log | head -5; exit 1; }
done
