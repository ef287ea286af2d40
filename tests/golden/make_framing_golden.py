#!/usr/bin/env python3
"""Generate the framing fixtures from the REFERENCE'S OWN writers and readers.

Runs only where /root/reference exists (this container).  `make -C oracle framing` compiles
db/value_log_writer.cc, db/value_log_reader.cc, db/log_writer.cc, db/log_reader.cc, table/table_builder.cc,
table/format.cc (+ their table/ and util/ dependencies and util/crc32c.cc) from their own source files into
oracle/_ref/ref_framing_golden, driven by tests/cpp/ref_framing_driver.cc.  This script runs it and commits:

  ref_framing.json   the driver's JSON (record layouts, stored header / trailer words, and what the reference
                     READERS return and report on intact and corrupted copies) + the SHA-256 of each written file
  ref_manifest.log   the MANIFEST-format log the reference log::Writer wrote (FIRST/MIDDLE/LAST fragments,
                     1/3/6-byte block trailers, a 0-byte FIRST fragment, a reopened writer appending mid-block)
  ref_table.sst      the SST the reference TableBuilder wrote (4 KiB blocks, 5-byte trailers)

The 3.4 MiB vlog (1,048,609-B records) is not committed: its payloads are the repo's splitmix64 stream (seed and
lengths in the JSON) and the reference's 8-byte headers plus the file's SHA-256 pin it completely.
"""
import hashlib
import json
import os
import subprocess
import tempfile

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_framing_golden")
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "framing"])
    with tempfile.TemporaryDirectory() as d:
        out = subprocess.run([DRIVER, d], check=True, capture_output=True, text=True).stdout
        j = json.loads(out)
        j["generator"] = "tests/golden/make_framing_golden.py (oracle/_ref/ref_framing_golden)"
        j["sha256"] = {}
        for name in ("vlog.bin", "manifest.log", "table.sst"):
            with open(os.path.join(d, name), "rb") as f:
                j["sha256"][name] = hashlib.sha256(f.read()).hexdigest()
        for src, dst in (("manifest.log", "ref_manifest.log"), ("table.sst", "ref_table.sst")):
            with open(os.path.join(d, src), "rb") as f, open(os.path.join(HERE, dst), "wb") as g:
                g.write(f.read())
    with open(os.path.join(HERE, "ref_framing.json"), "w") as f:
        json.dump(j, f, separators=(",", ":"))
    print("wrote ref_framing.json, ref_manifest.log, ref_table.sst")


if __name__ == "__main__":
    main()
