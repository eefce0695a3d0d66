"""Convert the reference's DBoW2 vocabulary (Examples/small_orb_omni_voc_9_6.yml, the
vocabulary the Lafida example loads, Examples/Lafida/mult_col_slam_lafida.cpp) into a compact
npz fixture under tests/golden/ so GPU tests can use it where /root/reference is absent.

The fixture is data only (node ids, parent ids, weights, 32-byte descriptors, word -> node),
parsed by mcs_amd.vocab.parse_yaml in file order.  Run in the build container:
    python tools/make_vocab_fixture.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multicol-slam-annotation_amd"))

from mcs_amd import vocab  # noqa: E402

SRC = "/root/reference/Examples/small_orb_omni_voc_9_6.yml"
DST = os.path.join(ROOT, "tests", "golden", "small_orb_omni_voc_9_6.npz")

if __name__ == "__main__":
    v = vocab.load_yaml(SRC)
    vocab.save_npz(DST, v)
    print("%s: k=%d L=%d scoring=%d weighting=%d nodes=%d words=%d -> %s (%d bytes)" % (
        SRC, v["k"], v["L"], v["scoring"], v["weighting"], len(v["node_id"]), len(v["word_node"]),
        DST, os.path.getsize(DST)))
