"""Parse the reference's Lafida settings / calibration YAML files (Examples/Lafida/*.yaml) with
mcs_amd.lafida.read_filestorage and store the key/value data as tests/golden/lafida_settings.json,
so CPU and GPU tests can run where /root/reference is absent.  Data only.
    python tools/make_lafida_fixture.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multicol-slam-annotation_amd"))

from mcs_amd import lafida  # noqa: E402

SRC = "/root/reference/Examples/Lafida"
DST = os.path.join(ROOT, "tests", "golden", "lafida_settings.json")

if __name__ == "__main__":
    out = {f: lafida.read_filestorage(os.path.join(SRC, f))
           for f in sorted(os.listdir(SRC)) if f.endswith(".yaml")}
    with open(DST, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print("%d files -> %s" % (len(out), DST))
