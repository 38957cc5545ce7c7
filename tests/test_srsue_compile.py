"""The drop-in boundary compiles srsUE unchanged: g++ -fsyntax-only of the reference's PHY worker (every DL
call site of SURVEY.md 8b) and of the MAC's DL HARQ entity (softbuffer ownership, dl_harq.cc:169-259) against
include/ (this repo's srslte/srslte.h, srslte/common/timestamp.h, srslte/utils/debug.h).  The only other
srsLTE headers srsUE includes -- the UHD glue (srslte/cuhd/cuhd.h, radio_uhd.h:29) and the MAC bit utilities
(srslte/utils/bit.h, mac/pdu.h) -- are not on the DL path and come from tests/c/srsue_stubs.  Needs the
reference tree (this container only; the GPU box has no /root/reference)."""
import os
import shutil
import subprocess

import pytest

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.isdir(REF) or shutil.which("g++") is None, reason="needs /root/reference and g++")
@pytest.mark.parametrize("src", ["ue/src/phy/phch_worker.cc", "ue/src/mac/dl_harq.cc"])
def test_srsue_source_compiles_against_include(src):
    cmd = ["g++", "-std=c++11", "-fsyntax-only", "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "tests", "c", "srsue_stubs"), "-I" + os.path.join(REF, "ue", "hdr"),
           "-I" + os.path.join(REF, "liblte", "hdr"), os.path.join(REF, src)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]


def test_stub_dir_holds_only_non_dl_srslte_headers():
    stubs = []
    for d, _, fs in os.walk(os.path.join(ROOT, "tests", "c", "srsue_stubs")):
        stubs += [os.path.relpath(os.path.join(d, f), os.path.join(ROOT, "tests", "c", "srsue_stubs")) for f in fs]
    assert sorted(stubs) == ["srslte/cuhd/cuhd.h", "srslte/utils/bit.h"]
