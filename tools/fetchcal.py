"""FETCH_SIZE / WRITE_SIZE per kernel of tools/micro/fetchcal against the bytes each one moved (VERDICT r5 item 3:
is the guide's FETCH_SIZE x2 right for k_step's dword scratch traffic?).
usage: python tools/fetchcal.py <fetch counter_collection.csv> <write counter_collection.csv> <out.json>"""
import csv
import json
import sys

GiB = 2 << 30
KNOWN = {  # kernel -> (bytes read, bytes written) by construction (fetchcal.hip)
    "k_fill": (0, GiB), "k_rd16": (GiB, 0), "k_wr4": (0, GiB), "k_rd4": (GiB, 0),
    "k_scratch": (16384 * 64 * 1024 * 4, 16384 * 64 * 1024 * 4),
}


def counter(path, name):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            k = r["Kernel_Name"].split("(")[0]
            out[k] = out.get(k, 0.0) + float(r["Counter_Value"]) * 1024.0  # KB -> bytes
    return out


def main():
    f, w = counter(sys.argv[1], "FETCH_SIZE"), counter(sys.argv[2], "WRITE_SIZE")
    rows = {}
    for k, (rd, wr) in KNOWN.items():
        rows[k] = {"bytes_read": rd, "bytes_written": wr, "fetch_size_bytes": f.get(k), "write_size_bytes": w.get(k),
                   "fetch_over_read": (f[k] / rd) if rd and k in f else None,
                   "write_over_written": (w[k] / wr) if wr and k in w else None}
    json.dump(rows, open(sys.argv[3], "w"), indent=1)
    for k, r in rows.items():
        print(k, {a: (round(b, 4) if isinstance(b, float) else b) for a, b in r.items()})


if __name__ == "__main__":
    main()
