"""CPU: the built library's rollout kernels keep their state in registers (round 5, VERDICT r4
#7).  The gfx950 code objects' metadata (scripts/kernel_resources.py) must show no scratch for
the flat-floor side kernels -- every mapping the bench's rollout, shard and config lines run --
so a change that brings a loop-invariant back into scratch (the 28-VGPR spill of rounds 3-4,
whose loads and write-backs were part of the excess HBM traffic) fails here, before any GPU run."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
LIB = os.path.join(ROOT, "ppo-bipedalwalker_amd", "libwk.so")


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/llvm/bin/clang-offload-bundler"),
                    reason="needs the built libwk.so and the ROCm LLVM tools")
def test_flat_floor_side_kernels_have_no_scratch():
    from kernel_resources import kernel_resources
    res = kernel_resources(LIB)
    # k_env_side<POLICY, RECORD, TRACE, Q, ROUGH>: the flat floor (ROUGH = false), both mappings
    side = {k: v for k, v in res.items() if k.startswith("_ZN2wk10k_env_side") and k.endswith("ELb0EEEvNS_9EnvParamsENS_8StepArgsE")}
    assert len(side) == 8, sorted(side)
    for k, (scratch, spilled, vgprs) in side.items():
        assert scratch == 0 and spilled == 0, (k, scratch, spilled)
    # the rollout kernel the bench times: the pair mapping with the policy and the recorder
    assert "_ZN2wk10k_env_sideILb1ELb1ELb0ELi1ELb0EEEvNS_9EnvParamsENS_8StepArgsE" in side
    # the update's gradient kernels: no scratch either (the ws gather's base formed in the loop)
    for k in ("_ZN2wk13k_ppo_grad_wsENS_8GradArgsE", "_ZN2wk13k_ppo_grad_tpILi1EEEvNS_8GradArgsE",
              "_ZN2wk13k_ppo_grad_tpILi2EEEvNS_8GradArgsE"):
        assert res[k][0] == 0, (k, res[k])
