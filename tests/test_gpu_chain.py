"""One frame stream chained through the whole hot path on the engine, as Tracking chains it
(tools/chain.py): ORB extraction of frame t -> SearchByProjection(motion) against frame t-1's
tracked map points -> the matched keypoints and their map points -> the object association of
frame t (src/Tracking.cc:1266-1281, 2434-2468), with LocalMapping's object maintenance at the
keyframes. The association consumes what the same step extracted and matched, not synthetic
observations. Engine and oracle each run the chain on their own outputs; every stage must agree
(keypoints, descriptors, match ids, the tracked map points handed on, detection outcomes, object
records) for 60 frames."""
import numpy as np
import pytest

import eao_accel as ea
import pyoracle as orc
from tools import chain

pytestmark = pytest.mark.gpu


def test_chained_stream_extract_match_associate():
    n = 60
    g = chain.run(chain.EngineBackend(ea), n)
    o = chain.run(chain.OracleBackend(orc), n)
    for t, (a, b) in enumerate(zip(g, o)):
        assert len(a["kps"]) == len(b["kps"]) and np.array_equal(a["kps"], b["kps"]), t
        assert np.array_equal(a["desc"], b["desc"]), t
        assert a["nmatch"] == b["nmatch"] and np.array_equal(a["match"], b["match"]), t
        assert np.array_equal(a["ids"], b["ids"]) and np.array_equal(a["boxes"], b["boxes"]), t
        assert np.array_equal(a["det"], b["det"]), (t, a["det"].tolist(), b["det"].tolist())
    # the chain exercises the path: map points carried by the matcher, and every association route
    assert sum(f["nmatch"] for f in g[1:]) > 200 * (n - 1)
    methods = {int(m) for f in g for m in f["det"][:, 0]}
    assert {1, 4, 5} <= methods  # IoU, projection, new objects
