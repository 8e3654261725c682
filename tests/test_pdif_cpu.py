"""pdif (RRUFF DIF + raw XY -> sample files), tools/pdif.cpp; parity with the reference
tutorial tool's output rules (tutorials/ann/file_dif.c:425-478).  Synthetic records:
the RRUFF database is not available offline."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PDIF = os.path.join(ROOT, "bin", "pdif")

DIF = """      Quartz   R040031
      Sample: T = {temp}
      CELL PARAMETERS:    4.9134    4.9134    5.4052   90.000   90.000  120.000
      SPACE GROUP: {sg}
               ATOM         X         Y         Z     OCCUPANCY  ISO(B)
                Si      0.4697    0.0000    0.0000    1.0000    0.5000
                 O      0.4135    0.2669    0.1191    1.0000    0.8000

            X-RAY WAVELENGTH:     {lam}
               2-THETA      INTENSITY    D-SPACING   H   K   L
                 20.86         22.07         4.2546   1   0   0
                 26.64        100.00         3.3435   1   0   1
"""
RAW = "##NAMES=x\n##END=\n4.0, 999\n5.5, 10\n12.0, 30\n20.9, 100\n26.6, 400\n50.0, 200\n89.9, 50\n"


@pytest.fixture(scope="module")
def pdif():
    if not os.path.exists(PDIF):
        subprocess.run(["make", "-C", ROOT, "-j8", "bin/pdif"], check=True, capture_output=True)
    return PDIF


def _record(d, name, **kw):
    p = dict(temp="25 C", sg="P3_221", lam="1.541838")
    p.update(kw)
    (d / "dif" / name).write_text(DIF.format(**p))
    (d / "raw" / name).write_text(RAW)


def test_pdif_sample_layout(pdif, tmp_path):
    for sub in ("dif", "raw", "samples"):
        (tmp_path / sub).mkdir()
    _record(tmp_path, "R1")
    _record(tmp_path, "R2", temp="300 K", sg="Fm-3m")
    _record(tmp_path, "R3", lam="0.710730")          # Mo radiation: skipped
    _record(tmp_path, "R4", sg="Xx9")                # unknown group: all -1
    r = subprocess.run([pdif, str(tmp_path), "-i", "4", "-o", "230", "-s", str(tmp_path / "samples")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "3 samples written, 1 records skipped" in r.stdout
    lines = (tmp_path / "samples" / "R1").read_text().split("\n")
    assert lines[0] == "[input] 5" and lines[2] == "[output] 230"
    vals = [float(v) for v in lines[1].split()]
    # T/273.15, then 4 bins of 21.25 deg in [5, 90): 140, 400, 200, 50 normalised by 400
    assert vals == pytest.approx([298.15 / 273.15, 0.35, 1.0, 0.5, 0.125], abs=1e-5)
    out = lines[3].split()
    assert len(out) == 230 and [i for i, v in enumerate(out) if v == "1.0"] == [153]   # P3_221 = 154
    l2 = (tmp_path / "samples" / "R2").read_text().split("\n")
    assert float(l2[1].split()[0]) == pytest.approx(300 / 273.15, abs=1e-5)
    assert [i for i, v in enumerate(l2[3].split()) if v == "1.0"] == [224]              # Fm-3m = 225
    assert not (tmp_path / "samples" / "R3").exists()
    assert "1.0" not in (tmp_path / "samples" / "R4").read_text().split("\n")[3].split()


def test_pdif_usage_errors(pdif, tmp_path):
    assert subprocess.run([pdif], capture_output=True).returncode == 1
    assert subprocess.run([pdif, str(tmp_path), "-i", "x", "-o", "3"], capture_output=True).returncode == 1
