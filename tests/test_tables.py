"""Curve constants and the base-point table are generated from the curve
definition (tools/gen_tables.py); check them against the reference's
literal tables when the reference tree is present."""
import os
import re
import subprocess
import sys

import pytest

from conftest import ROOT

REF = "/root/reference/src/ballet/ed25519"
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_tables  # noqa: E402


def _ints(txt):
    return [int(x) for x in re.findall(r"-?\d+", txt)]


def test_generated_headers_up_to_date(tmp_path):
    before = {f: open(os.path.join(ROOT, f)).read() for f in
              ("oracle/fd_ed25519_oracle_tables.h", "firedancer_amd/csrc/fd_ed25519_tables.h")}
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_tables.py")], check=True)
    for f, txt in before.items():
        assert open(os.path.join(ROOT, f)).read() == txt, f


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_constants_match_reference():
    ge = open(os.path.join(REF, "avx", "fd_ed25519_ge.c")).read()
    d = _ints(re.search(r"d\[1\] = \{\{\s*\{([^}]*)\}", ge).group(1))
    sqrtm1 = _ints(re.search(r"sqrtm1\[1\] = \{\{\s*\{([^}]*)\}", ge).group(1))
    assert d == gen_tables.limbs(gen_tables.D)
    assert sqrtm1 == gen_tables.limbs(gen_tables.SQRTM1)
    blk = re.search(r"l111d2\[40\][^{]*\{(.*?)\};", ge, re.S).group(1)
    vals = [int(x) for x in re.findall(r"\(long\)\(uint\)\s*(-?\d+)", blk)]
    assert vals == gen_tables.limbs(2 * gen_tables.D)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_bi_precomp_matches_reference():
    txt = open(os.path.join(REF, "table", "fd_ed25519_ge_bi_precomp.c")).read()
    body = txt[txt.index("bi_precomp[8][1] = {"):]
    rows = re.findall(r"\{\{\{([^}]*)\}\}\}", body)
    assert len(rows) == 24
    ref = [_ints(r) for r in rows]
    gen = gen_tables.base_multiples()
    for i, (ypx, ymx, xy2d) in enumerate(gen):
        assert ref[3 * i] == ypx and ref[3 * i + 1] == ymx and ref[3 * i + 2] == xy2d, i
