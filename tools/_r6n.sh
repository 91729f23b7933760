# the full GPU tier, then the driver's bench command (N=1), as at round end
bash tools/gpu_steps.sh "tests r6n_tier" "driver r6n_drv"
