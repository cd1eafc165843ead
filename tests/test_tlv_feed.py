"""fuzzer_tlv_server's InsertTestcase deserialisation: the
packet chunks this repository's module derives from a testcase
(TlvServer::TestcaseFeed: the canonical JSON parsed straight into the Feed
layout, anything else through the general parser) must equal what the
reference's nlohmann-based Deserialize gives (fuzzer_tlv_server.cc:36-40,
67-75), on the committed fixtures (tests/golden/gen_tlv_feed_fixtures.py, from
oracle/_ref/ref_hostcheck) and, when the reference build is present, live on
mutator output."""
import json
import os
import random

import pytest

from tests.golden.gen_tlv_feed_fixtures import canonical, feeds, packet

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
from tests.cpu_bins import HOSTCHECK as OURS  # noqa: E402
REF = os.path.join(ROOT, "oracle", "_ref", "ref_hostcheck")

pytestmark = pytest.mark.skipif(not os.path.exists(OURS), reason="oracle/hostcheck not built")


def load():
    with open(os.path.join(HERE, "golden", "tlv_feed_fixtures.json")) as f:
        return json.load(f)["cases"]


def test_feeds_match_reference_fixtures():
    cases = load()
    got = feeds(OURS, [bytes.fromhex(c["tc"]) for c in cases])
    bad = [(i, c["tc"][:80]) for i, (c, g) in enumerate(zip(cases, got)) if g != c["feed"]]
    assert not bad, f"{len(bad)} of {len(cases)} differ, first: {bad[:4]}"
    assert sum(1 for c in cases if c["feed"] is None) >= 20  # the rejections are covered too


@pytest.mark.skipif(not os.path.exists(REF), reason="oracle/_ref/ref_hostcheck not built")
def test_feeds_match_reference_live_on_large_packets():
    rng = random.Random(77)
    tcs = [canonical([packet(rng, 1200) for _ in range(rng.randint(1, 10))]) for _ in range(400)]
    tcs += [t[:rng.randint(0, len(t))] for t in tcs[:100]]
    assert feeds(OURS, tcs) == feeds(REF, tcs)


def test_mutator_handoff_feed_equals_parsed_feed():
    """PrepareInsert takes the feed the tlv mutator built with the testcase
    (no JSON parse) when the bytes are the mutator's last output: over a
    growing corpus, that feed and a truncated copy's (parsed) equal
    TestcaseFeed's parse of the same bytes."""
    import subprocess
    out = subprocess.run([OURS, "tlv-prep", "7", "20000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.split() == ["P", "20000", "0"]
