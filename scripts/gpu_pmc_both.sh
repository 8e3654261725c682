cd "${GRAFT_REPO_ROOT}"
PMC_TAG=_mnist bash scripts/pmc_step.sh > /dev/null 2>&1 || exit $?
PMC_TAG=_rruff bash scripts/pmc_step.sh --model rruff > /dev/null 2>&1 || exit $?
cat gpurun_out/pmc_step_mnist.txt gpurun_out/pmc_step_rruff.txt
