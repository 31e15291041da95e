#!/usr/bin/env python3
"""Regenerate tests/golden/snap_cases.json: .net texts read by the REFERENCE's own
SNAPReader (readerwriter.h:78-90, `stream >> X` then `stream >> Y`, compiled from
/root/reference into oracle/_ref/ref_harness `snap` mode).  Build container only."""
import json
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")

CASES = [
    "1 2\n3 4\n5 6\n",
    "1 2\n3 4\n5",                                   # incomplete last pair
    "  10\t20\r\n30    40\r\n\n\n50 60",             # tabs, CRLF, blank lines
    "1 2\n3 x\n5 6\n",                               # a token that is no number
    "1 2\n4294967295 0\n4294967296 1\n7 8\n",        # u32 overflow
    "3 4x\n5 6\n",                                   # trailing junk after a number
    "1 2\n3 4#5\n6 7\n",
    "+5 7\n8 9\n",                                   # explicit sign
    "-1 2\n3 4\n",                                   # negative: wraps modulo 2^32
    "00000000000000000007 1\n2 3\n",                 # leading zeros
    "1 2\n# comment 3 4\n5 6\n",                     # '#' is just a bad token to SNAPReader
    "",
    "\n \n",
    "7\t8\f9\v10\n",
]


def main():
    out = []
    with tempfile.TemporaryDirectory() as td:
        for i, text in enumerate(CASES):
            path = os.path.join(td, f"c{i}.net")
            open(path, "w").write(text)
            r = subprocess.run([HARNESS, "snap", path], check=True, capture_output=True, text=True).stdout
            pairs = [[int(x) for x in ln.split()] for ln in r.splitlines()]
            out.append({"text": text, "pairs": pairs})
    json.dump(out, open(os.path.join(HERE, "snap_cases.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
