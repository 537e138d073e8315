"""The C ABI (include/sat_hip.h) without a GPU: the library loads, exports every declared
entry point, and the ctypes mirrors of its structs match the C layout (checked by compiling
a probe with gcc against the same header)."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "sat_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sat_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    import sat_amd
    lib = sat_amd._lib.lib()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert lib.sat_abi_version() == 1
    assert set(declared_functions()) == set(sat_amd._lib.EXPORTED)


def test_error_strings():
    import sat_amd
    lib = sat_amd._lib.lib()
    assert lib.sat_error_string(0) == b"success"
    assert b"invalid" in lib.sat_error_string(9001)


def test_struct_layouts_match_c(tmp_path):
    import sat_amd
    L = sat_amd._lib
    probe = tmp_path / "probe.c"
    probe.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "sat_hip.h"
#define P(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("SatGemmArgs %zu\nSatDecoderDims %zu\nSatDecoderLayout %zu\nSatConvGeom %zu\n",
         sizeof(SatGemmArgs), sizeof(SatDecoderDims), sizeof(SatDecoderLayout), sizeof(SatConvGeom));
  P(SatGemmArgs, B) P(SatGemmArgs, C) P(SatGemmArgs, alpha) P(SatGemmArgs, bias) P(SatGemmArgs, add1)
  P(SatGemmArgs, act) P(SatGemmArgs, aux) P(SatGemmArgs, aux_dtype)
  P(SatDecoderDims, dtype) P(SatDecoderDims, seed) P(SatDecoderDims, seed_ptr) P(SatDecoderDims, split_target)
  P(SatDecoderLayout, do_b) P(SatDecoderLayout, total)
  return 0;
}
''')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.dirname(HEADER), str(probe), "-o", str(exe)], check=True)
    out = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                        check=True).stdout.splitlines())
    assert int(out["SatGemmArgs"]) == ctypes.sizeof(L.SatGemmArgs)
    assert int(out["SatDecoderDims"]) == ctypes.sizeof(L.SatDecoderDims)
    assert int(out["SatDecoderLayout"]) == ctypes.sizeof(L.SatDecoderLayout)
    assert int(out["SatConvGeom"]) == ctypes.sizeof(L.SatConvGeom)
    for key, val in out.items():
        if "." in key:
            struct, field = key.split(".")
            assert getattr(getattr(L, struct), field).offset == int(val), key
