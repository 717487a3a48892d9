#!/usr/bin/env python3
"""Resources (VGPR / SGPR / scratch / occupancy) of the run-time compiled
butterfly kernel for one decoder, compiled here exactly as cvd_rtc.cpp does it
(device-only clang, same flags), with optional -D tuning defines:

  python3 spec_resource.py [m6|m2|...] [-DCVD_K1B_WAVES=5 ...] [--isa out.s]

(-DCVD_K1B_BITSLICE=1: the bit-sliced m = 6 form, k1s, as cvd_rtc.cpp builds it for models
with bit-sliced tables)

No GPU needed: the code constant (out(j, 0) of every butterfly) comes from the
host tables (cvd_code_tables), as build_bfly computes it.
"""
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def code_constant(cfg):
    from __graft_entry__ import load_package
    pkg = load_package()
    cc = pkg.CONFIG_CODES[cfg]
    out, _ = pkg.Code(cc["gen1"], cc["m"], cc["k"], cc["n"]).tables()
    return cc["m"], sum(int(out[j, 0]) << (2 * j) for j in range((1 << cc["m"]) // 2))


def main():
    args = sys.argv[1:]
    isa = None
    if "--isa" in args:
        i = args.index("--isa")
        isa = args[i + 1]
        del args[i:i + 2]
    defs = [x for x in args if x.startswith("-")]   # -D... and -mllvm pairs (as CVD_JIT_DEFINES)
    rest = [x for x in args if not x.startswith("-")]
    m, xm = code_constant(rest[0] if rest else "m6")
    clang = os.environ.get("CVD_JIT_CLANG", "/opt/rocm/lib/llvm/bin/clang++")
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "k1b_spec.hip")
        with open(src, "w") as f:
            f.write('#include <hip/hip_runtime.h>\n#include "cvd_device.h"\n'
                    'extern "C" __global__ __launch_bounds__(cvd_dev::kK1bBlock, cvd_dev::kK1bWavesPerSimd)\n'
                    f'void cvd_k1b_spec(cvd_dev::ExpArgs a) {{ cvd_dev::k1b_spec_entry<{m}, 0x{xm:016x}ull>(a); }}\n'
                    'extern "C" __global__ __launch_bounds__(cvd_dev::kK1bBlock, cvd_dev::kK1bWavesPerSimd)\n'
                    f'void cvd_k1b_spec_multi(cvd_dev::MultiArgs a) {{ cvd_dev::k1b_spec_multi_entry<{m}, 0x{xm:016x}ull>(a); }}\n')
        base = [clang, "-x", "hip", "--offload-arch=gfx950", "--offload-device-only", "--no-gpu-bundle-output",
                "-O3", "-std=c++17", "-ffp-contract=off", "-mllvm", "--amdgpu-sched-strategy=max-ilp",
                "-I", HERE, *defs]
        r = subprocess.run(base + ["-Rpass-analysis=kernel-resource-usage", "-c", src, "-o",
                                   os.path.join(d, "k.co")], capture_output=True, text=True)
        for line in r.stderr.splitlines():
            if "remark" in line or "error" in line:
                print(line.split("remark: ")[-1])
        if r.returncode:
            sys.exit(r.returncode)
        if isa:
            subprocess.run(base + ["-S", src, "-o", isa], check=True)
            print("ISA written to", isa)


if __name__ == "__main__":
    main()
