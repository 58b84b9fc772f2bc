"""Generate tests/golden/tables.json from the reference's literal GF(2^8) tables.

Runs only in the build container, where /root/reference exists.  It reads
KRS/galois.go as text (vendor/github.com/klauspost/reedsolomon/galois.go:28-937),
extracts the integer literals of each table and records their length and the
SHA-256 of their byte serialisation.  Nothing of the reference's source is
stored: only the digests, which tests/test_oracle.py compares against the
oracle's regenerated tables.

    python tests/golden/make_table_fixture.py
"""
import hashlib
import json
import os
import re
import sys

REF = "/root/reference/vendor/github.com/klauspost/reedsolomon/galois.go"
TABLES = {
    # name: (element width in bytes)
    "logTable": 1,
    "expTable": 1,
    "invTable": 1,
    "mulTable": 1,
    "mulTableLow": 1,
    "mulTableHigh": 1,
    "gf2p811dMulMatrices": 8,
}


def extract(src: str, name: str):
    m = re.search(r"var\s+%s\s*=\s*[^{]*\{" % re.escape(name), src)
    if not m:
        raise KeyError(name)
    i = m.end()
    depth = 1
    j = i
    while depth:
        ch = src[j]
        if ch == "{":
            depth += 1
        elif ch == "}":
            depth -= 1
        j += 1
    body = src[i : j - 1]
    return [int(t, 0) for t in re.findall(r"0x[0-9a-fA-F]+|\d+", body)]


def main():
    if not os.path.exists(REF):
        sys.exit("reference not present; fixture must be generated in the build container")
    src = open(REF).read()
    out = {"source": "vendor/github.com/klauspost/reedsolomon/galois.go (v1.11.7)", "tables": {}}
    for name, width in TABLES.items():
        vals = extract(src, name)
        blob = b"".join(v.to_bytes(width, "little") for v in vals)
        out["tables"][name] = {"count": len(vals), "width": width,
                               "sha256": hashlib.sha256(blob).hexdigest()}
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tables.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
