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
    assert lib.sat_abi_version() == sat_amd._lib.ABI_VERSION == header_abi_version() == 9
    assert set(declared_functions()) == set(sat_amd._lib.EXPORTED)


def header_abi_version():
    return int(re.search(r"#define SAT_ABI_VERSION (\d+)", open(HEADER).read()).group(1))


def test_no_process_global_tuning_state():
    """Kernel selection is a per-call argument (SatPolicy), not process-global state: the header
    declares no setter / mode / experiment hook, and the library exports none."""
    import sat_amd
    names = declared_functions()
    bad = [f for f in names if re.search(r"_set_|_mode\b|experiment|cu_mask|trace", f)]
    assert not bad, bad
    exported = subprocess.run(["nm", "-D", "--defined-only", sat_amd._lib.LIB_PATH], capture_output=True,
                              text=True, check=True).stdout
    syms = re.findall(r" T (sat_\w+)", exported)
    assert sorted(syms) == names, sorted(set(syms) ^ set(names))
    text = open(HEADER).read()
    assert "SatPolicy* policy" in text.replace("const SatPolicy", "SatPolicy")


def test_library_refuses_other_abi_version(monkeypatch):
    import sat_amd
    L = sat_amd._lib
    monkeypatch.setattr(L, "_lib", None)
    monkeypatch.setattr(L, "ABI_VERSION", 3)
    with pytest.raises(RuntimeError, match="C-ABI version"):
        L.lib()
    monkeypatch.undo()
    assert L.lib().sat_abi_version() == L.ABI_VERSION == 9


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
  printf("SatGemmArgs %zu\nSatDecoderDims %zu\nSatDecoderLayout %zu\nSatConvGeom %zu\nSatPolicy %zu\n",
         sizeof(SatGemmArgs), sizeof(SatDecoderDims), sizeof(SatDecoderLayout), sizeof(SatConvGeom),
         sizeof(SatPolicy));
  P(SatGemmArgs, B) P(SatGemmArgs, C) P(SatGemmArgs, alpha) P(SatGemmArgs, bias) P(SatGemmArgs, add1)
  P(SatGemmArgs, act) P(SatGemmArgs, aux) P(SatGemmArgs, aux_dtype) P(SatGemmArgs, policy)
  P(SatDecoderDims, dtype) P(SatDecoderDims, seed) P(SatDecoderDims, seed_ptr) P(SatDecoderDims, split_target)
  P(SatDecoderDims, policy) P(SatPolicy, attn_bwd) P(SatPolicy, decoder_splits) P(SatPolicy, split_gemm) P(SatPolicy, split_k) P(SatPolicy, stamps)
  P(SatPolicy, stamp_capacity) P(SatGemmArgs, workspace) P(SatGemmArgs, workspace_bytes)
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
    assert int(out["SatPolicy"]) == ctypes.sizeof(L.SatPolicy)
    for key, val in out.items():
        if "." in key:
            struct, field = key.split(".")
            assert getattr(getattr(L, struct), field).offset == int(val), key
