# Round-3 (sq2): SQ counters of the bench kernels for the final library
tools/gpu_steps.sh "sqbench:::300:::bash tools/gpu_sq_bench.sh"
