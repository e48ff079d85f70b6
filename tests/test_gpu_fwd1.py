"""GPU parity of the experimental one-wave-per-SIMD forward (vb_attn_fwd1.hip, selected with
VB_FWD1=1; profiles/r04_fwd1_experiments.md). The library reads the switch once per process, so the
checks run in one child process: the forward's own parity cases (dense vs oracle, pooled branch,
forced rescales at scores 100-300 log2 units above the first tile's max, the full-size module vs
the oracle) at both head dims."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fwd1_parity_in_child_process():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, VB_FWD1="1")
    sel = ("test_dense_matches_oracle_and_sdpa or test_huge_late_scores or test_fused_pooled_branch "
           "or test_full_size_module_against_oracle or test_module_matches_reference_e2e_golden")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_forward.py"),
                        os.path.join(ROOT, "tests", "test_gpu_module.py"), "-k", sel],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert " passed" in r.stdout and "failed" not in r.stdout, tail
