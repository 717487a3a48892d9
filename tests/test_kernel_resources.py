"""The run-time compiled m = 6 detector kernel (cvd_k1b_spec) must keep its
register budget: no scratch (spills to memory in the step loop cost ~30% of the
launch, measured when a cursor change tipped the allocator over), and 4 waves
per SIMD.  Compiled here exactly as the JIT does (csrc/spec_resource.py); no GPU.
Every variant upload_model builds by default is checked: the butterfly kernel, and the
bit-sliced kernel k1s with the pre-filter (1,024-thread blocks, the lockstep p), with the
128-KiB LDS filter (walking models) and with neither (CVD_BS_PF=0)."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPEC = os.path.join(ROOT, "detecting-convolutional-codes-via-markovian-statistics_amd", "csrc", "spec_resource.py")

VARIANTS = {
    "butterfly": [],
    # the butterfly kernel on a walking model's 128-KiB LDS filter in 1,024-thread blocks: what
    # a model sized for k1s runs if its bit-sliced JIT build fails
    "butterfly_ldsf_1024": ["-DCVD_K1B_LDSF=1", "-DCVD_K1B_BLOCK=1024", "-DCVD_FILTER_PAT_BITS=10"],
    "k1s_pf": ["-DCVD_K1B_BITSLICE=1", "-DCVD_K1S_PF=1", "-DCVD_K1B_BLOCK=1024", "-DCVD_FILTER_PAT_BITS=10"],
    "k1s_ldsf": ["-DCVD_K1B_BITSLICE=1", "-DCVD_K1B_LDSF=1", "-DCVD_K1B_BLOCK=1024", "-DCVD_FILTER_PAT_BITS=10"],
    "k1s_global": ["-DCVD_K1B_BITSLICE=1"],
    # three-line directory slots (CVD_BS_SLOT3=1, measured and not the default: profiles/r06j)
    "k1s_pf_slot3": ["-DCVD_K1B_BITSLICE=1", "-DCVD_K1S_PF=1", "-DCVD_K1B_BLOCK=1024", "-DCVD_FILTER_PAT_BITS=10",
                     "-DCVD_K1S_SLOT3=1"],
    # the select-form ACS and compare-form cursor (CVD_BS_ETAB2=0, CVD_K1S_AMASK=0: the forms before
    # round 6's VALU cuts, kept for A/Bs)
    "k1s_pf_select_forms": ["-DCVD_K1B_BITSLICE=1", "-DCVD_K1S_PF=1", "-DCVD_K1B_BLOCK=1024",
                            "-DCVD_FILTER_PAT_BITS=10", "-DCVD_BS_ETAB2=0", "-DCVD_K1S_AMASK=0"],
    # the two-step lookup pipeline (CVD_K1S_DEEP=2, measured and not the default: profiles/r06u)
    "k1s_pf_deep2": ["-DCVD_K1B_BITSLICE=1", "-DCVD_K1S_PF=1", "-DCVD_K1B_BLOCK=1024", "-DCVD_FILTER_PAT_BITS=10",
                     "-DCVD_K1S_DEEP=2"],
}


@pytest.mark.skipif(not shutil.which("/opt/rocm/lib/llvm/bin/clang++"), reason="ROCm clang not present")
@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_spec_kernel_no_scratch_4_waves(variant):
    out = subprocess.run([sys.executable, SPEC, "m6", *VARIANTS[variant]], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    # both entries (one model per launch, and the multi-model entry)
    scratch = [int(x) for x in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", out.stdout)]
    occ = [int(x) for x in re.findall(r"Occupancy \[waves/SIMD\]: (\d+)", out.stdout)]
    assert len(scratch) == 2 and all(s == 0 for s in scratch), out.stdout
    assert len(occ) == 2 and all(o >= 4 for o in occ), out.stdout
