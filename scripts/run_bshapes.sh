TESTS="${T_:-tests/test_gpu_baseline_shapes.py}" LOGNAME_=bshapes TLIMIT=600 bash scripts/gpu_tests.sh; tail -40 gpurun_out/bshapes.log
