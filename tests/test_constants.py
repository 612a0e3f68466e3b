"""The product's constant tables (neptune-core_amd/csrc/tip5_constants.h) against the
oracle's independent derivation (BLAKE3 round constants, cubic lookup table, MDS column)."""
import os
import re

import tip5_ref as T

HDR = os.path.join(os.path.dirname(__file__), "..", "neptune-core_amd", "csrc", "tip5_constants.h")


def _array(name, src):
    m = re.search(name + r"\[\d+\]\s*=\s*\{(.*?)\};", src, re.S)
    return [int(x.strip().rstrip("ull"), 0) for x in m.group(1).replace("\n", " ").split(",") if x.strip()]


def test_header_constants_match_oracle():
    src = open(HDR).read()
    assert _array("TIP5_RC_RAW", src) == [T.to_mont(c) for c in T.ROUND_CONSTANTS]
    assert _array("TIP5_LUT", src) == T.LOOKUP_TABLE
    assert _array("TIP5_MDS", src) == T.MDS_FIRST_COLUMN
