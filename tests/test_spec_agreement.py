"""The product's spec header and the oracle's spec header were written separately;
they must agree on every constant of the restated relab/bbhash + FNV algorithm."""
import os
import re

from conftest import ROOT


def _read(p):
    return open(os.path.join(ROOT, p)).read()


def _c_int(s):
    s = s.rstrip("uUlL")
    return int(s, 16) if s.lower().startswith("0x") else int(s)


def test_constants_agree():
    orc = _read("oracle/bbhash_oracle_spec.h")
    prod = _read("s3-inv-db_amd/csrc/bbhash_spec.h")

    def o(name):
        return _c_int(re.search(rf"#define {name} (\S+)", orc).group(1))

    def p(name):
        return _c_int(re.search(rf"constexpr \w+ {name} = ([0-9a-fA-Fx]+)", prod).group(1))

    assert o("ORC_FNV_OFFSET64") == p("kFnvOffset")
    assert o("ORC_FNV_PRIME64") == p("kFnvPrime")
    assert o("ORC_HASH_M") == p("kHashM")
    assert o("ORC_MIX_MUL") == p("kMixMul")
    assert o("ORC_GAMMA_NUM") == p("kGammaNum")
    assert o("ORC_MAX_LEVELS") == p("kMaxLevels")
    assert o("ORC_MARSHAL_PARTITION_HDR") == p("kPartitions")
