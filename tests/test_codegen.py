"""Code-generation guards on the built gfx950 library (CPU: disassembly only).

The pair kernels' f32 epilogue compiled with packed-f32 VALU ops
(v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32, made by the SLP vectorizer) gave
timing-dependent wrong d/D'/r2 on MI355X (one accumulator row of the one-plane
kernel, lanes 48-63).  The Makefile builds with
-fno-slp-vectorize; this test fails if any packed-f32 op reaches the shipped
code objects again."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

from weightedld_amd import _lib

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump absent")
def test_no_packed_f32_valu_ops():
    assert os.path.exists(_lib.LIB_PATH), _lib.LIB_PATH
    with tempfile.TemporaryDirectory() as td:
        lib = os.path.join(td, "lib.so")
        shutil.copy(_lib.LIB_PATH, lib)
        subprocess.run([OBJDUMP, "--offloading", lib], cwd=td, check=True, capture_output=True)
        cos = [os.path.join(td, f) for f in os.listdir(td) if f.endswith("gfx950")]
        assert cos, "no gfx950 code objects in " + _lib.LIB_PATH
        kernels = 0
        for co in cos:
            dis = subprocess.run([OBJDUMP, "-d", co], check=True, capture_output=True, text=True).stdout
            kernels += len(re.findall(r"^[0-9a-f]+ <_Z\w*kernel\w*>:", dis, re.M))
            bad = re.findall(r"v_pk_(?:add|mul|fma)_f32\b.*", dis)
            assert not bad, (os.path.basename(co), len(bad), bad[:3])
        assert kernels > 10, kernels
