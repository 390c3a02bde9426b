"""Turn the reference's own fr3_long_office inputs into a committed fixture.

Run HERE only (it reads /root/reference, which does not exist on the GPU box):

    python tools/make_fr3_inputs.py  ->  tests/golden/fr3_inputs.npz

What it reads (data files, not code):
  * data/rgb_full_demo.txt, data/rgb_seq_pose.txt -- image lists; mono_tum's LoadImages
    skips 6 lines (3 header lines + the first 3 images, Examples/Monocular/mono_tum.cc:136-144),
    giving 2582 ("Full") and 405 (the demo flags) frames;
  * data/yolo_txts.tar.gz -- per-frame YOLO boxes, read the way Tracking::GrabImageMonocular
    does (src/Tracking.cc:426-469): "./data/yolo_txts/" + to_string(timestamp) + ".txt", each
    line parsed with `int tmp; istr >> tmp` -- the score "0.824041" yields 0 and stops the
    line, so every m_score is 0 and the stable sort by score keeps file order;
  * data/groundtruth.txt -- TUM poses (t tx ty tz qx qy qz qw, camera-to-world), looked up
    per frame as src/Tracking.cc:508-554 does: the first row whose to_string(t) minus its
    last 4 characters equals the frame's (a match on the first two decimals, string-truncated).

Stored per frame (Full list order): timestamp, the matched GT row (or NaN when the
reference's lookup finds none) and the boxes [class, x, y, w, h] in file order.
"""
import io
import os
import tarfile

import numpy as np

REF = "/root/reference/data"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_images(path):
    """mono_tum.cc:131-165: skip 6 lines, then `ss >> t` per non-empty line."""
    lines = open(path).read().split("\n")[6:]
    return [float(s.split()[0]) for s in lines if s]


def cpp_int_tokens(line):
    """`while (istr >> tmp)` with int tmp: read whitespace-separated integers until
    a token does not start with an integer; a token like "0.82" yields 0 and stops."""
    out = []
    for tok in line.split():
        i = 0
        if i < len(tok) and tok[i] in "+-":
            i += 1
        j = i
        while j < len(tok) and tok[j].isdigit():
            j += 1
        if j == i:
            break
        out.append(int(tok[:j]))
        if j != len(tok):
            break
    return out


def to_string(x):
    return "%f" % x  # std::to_string(double) is "%f"


def main():
    full = load_images(os.path.join(REF, "rgb_full_demo.txt"))
    demo = load_images(os.path.join(REF, "rgb_seq_pose.txt"))
    tf = tarfile.open(os.path.join(REF, "yolo_txts.tar.gz"))
    files = {os.path.basename(m.name): m for m in tf.getmembers() if m.isfile()}
    gt_lines = open(os.path.join(REF, "groundtruth.txt")).read().split("\n")[3:]
    gt = [[float(v) for v in l.split()] for l in gt_lines if l.strip()]
    gt_keys = [to_string(r[0])[:-4] for r in gt]
    first = {}
    for k, key in enumerate(gt_keys):
        first.setdefault(key, k)
    ts, gtrow, boff, boxes = [], [], [0], []
    for t in full:
        name = to_string(t) + ".txt"
        if name not in files:
            raise SystemExit("yolo_detection file open fail: " + name)  # Tracking.cc:427-431
        rows = [cpp_int_tokens(l) for l in io.TextIOWrapper(tf.extractfile(files[name])).read().split("\n")]
        rows = [r for r in rows if r]  # getline of an empty last line pushes an empty row; never read
        for r in rows:
            assert len(r) == 6 and r[5] == 0, (name, r)  # class x y w h score(=0, Q1)
            boxes.append(r[:5])
        boff.append(len(boxes))
        ts.append(t)
        k = first.get(to_string(t)[:-4])
        gtrow.append(gt[k][1:8] if k is not None else [np.nan] * 7)
    ts = np.asarray(ts, np.float64)
    # the replay needs a pose for every frame; where the reference's lookup finds no
    # row (gaps in the 100 Hz GT) the harness interpolates between the bracketing GT
    # rows: translation linearly, quaternion by normalised lerp (sign-aligned)
    G = np.asarray(gt, np.float64)
    pose = np.zeros((len(ts), 7))
    for i, t in enumerate(ts):
        if np.isfinite(gtrow[i][0]):
            pose[i] = gtrow[i]
            continue
        j = int(np.searchsorted(G[:, 0], t))
        j = min(max(j, 1), len(G) - 1)
        a, b = G[j - 1], G[j]
        w = float(np.clip((t - a[0]) / (b[0] - a[0]), 0.0, 1.0))
        qa, qb = a[4:8], b[4:8] * (1.0 if np.dot(a[4:8], b[4:8]) >= 0 else -1.0)
        q = (1 - w) * qa + w * qb
        pose[i, :3] = (1 - w) * a[1:4] + w * b[1:4]
        pose[i, 3:] = q / np.linalg.norm(q)
    demo_first = int(np.nonzero(ts == demo[0])[0][0]) if demo[0] in set(full) else -1
    if demo_first >= 0:
        assert np.array_equal(ts[demo_first:demo_first + len(demo)], np.asarray(demo)), "demo list is a slice"
    out = os.path.join(ROOT, "tests", "golden", "fr3_inputs.npz")
    np.savez_compressed(out, timestamps=ts, gt=np.asarray(gtrow, np.float64), pose=pose,
                        box_off=np.asarray(boff, np.int32), boxes=np.asarray(boxes, np.int16),
                        demo_timestamps=np.asarray(demo, np.float64), demo_first=np.int32(demo_first))
    nm = int(np.isfinite(np.asarray(gtrow)[:, 0]).sum())
    print("%d frames (%d demo), %d boxes, GT matched for %d frames -> %s" % (len(ts), len(demo), len(boxes), nm, out))


if __name__ == "__main__":
    main()
