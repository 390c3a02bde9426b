"""Fixtures pinning the line-detector restatement (oracle/lines_ref.cpp) against the Edge Drawing
library's own held outputs -- DATA only, read from the reference tree, never executed:
  Thirdparty/EDTest/lena.pgm + ED-EdgeMap.pgm: the edge map EDTest/main.cpp:57-74 saved from
      DetectEdgesByED(lena, SOBEL_OPERATOR, 36, 8, 1.0) (every segment pixel set to 255);
  Thirdparty/EDLines/house.pgm + EDLinesTest/LineSegments.txt (inside EDLinesTest-x64.tar.gz):
      the 168 segments EDLines/main.cpp:46-75 printed ("%6.2lf") from DetectLinesByED(house).
Writes tests/golden/ed_pin.npz. The prebuilt EDLib.a / EDLinesLib.a / EDLinesTest binaries are
never run or loaded."""
import os
import re
import sys
import tarfile

import numpy as np

REF = "/root/reference/Thirdparty"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "ed_pin.npz")


def read_pgm(data):
    toks, i = [], 0
    while len(toks) < 4:
        while data[i:i + 1].isspace():
            i += 1
        if data[i:i + 1] == b"#":
            while data[i:i + 1] != b"\n":
                i += 1
            continue
        j = i
        while not data[j:j + 1].isspace():
            j += 1
        toks.append(data[i:j])
        i = j
    assert toks[0] == b"P5" and toks[3] == b"255"
    w, h = int(toks[1]), int(toks[2])
    i += 1  # the single whitespace after maxval
    return np.frombuffer(data[i:i + w * h], np.uint8).reshape(h, w).copy()


def main():
    lena = read_pgm(open(os.path.join(REF, "EDTest", "lena.pgm"), "rb").read())
    edmap = read_pgm(open(os.path.join(REF, "EDTest", "ED-EdgeMap.pgm"), "rb").read())
    house = read_pgm(open(os.path.join(REF, "EDLines", "house.pgm"), "rb").read())
    with tarfile.open(os.path.join(REF, "EDLines", "EDLinesTest-x64.tar.gz")) as t:
        txt = t.extractfile("EDLinesTest/LineSegments.txt").read().decode("ascii")
    rows = [l for l in txt.splitlines()[1:] if l.strip()]
    segs = np.array([[float(v) for v in re.findall(r"-?\d+\.\d+", l)] for l in rows], np.float64)
    assert segs.shape == (168, 4), segs.shape
    assert set(np.unique(edmap)) <= {0, 255}
    np.savez_compressed(OUT, lena=lena, ed_edge_map=np.packbits(edmap > 0), house=house, ed_segments=segs)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    sys.exit(main())
