"""Join tools/fetch_calib's known byte counts with its rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; kB per
dispatch) into a calibration table: factor = known bytes / counted bytes per access pattern.

    python tools/fetch_calib.py <known.json> <fetch_pass_dir> <write_pass_dir> > profiles/<round>/fetch_calibration.json
"""
import csv
import glob
import json
import sys


def counters(d):
    path = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    out = {}
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"]
        key = ("k_store8" if "k_store<unsigned long>" in name else "k_store4" if "k_store<unsigned int>" in name
               else name.split("(")[0].split()[-1])
        out.setdefault(key, []).append(float(row["Counter_Value"]))
    return out


def main():
    known = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["known"]
    fetch, write = counters(sys.argv[2]), counters(sys.argv[3])
    table = {}
    for k, kb in known.items():
        f = fetch.get(k, [None])
        w = write.get(k, [None])
        fk = f[-1] * 1024.0 if f[-1] is not None else None  # FETCH_SIZE / WRITE_SIZE are in kB
        wk = w[-1] * 1024.0 if w[-1] is not None else None
        table[k] = {"known_read": kb["read"], "known_write": kb["write"], "fetch_size_bytes": fk,
                    "write_size_bytes": wk,
                    "read_factor": kb["read"] / fk if fk and kb["read"] else None,
                    "write_factor": kb["write"] / wk if wk and kb["write"] else None}
    print(json.dumps({"device": "MI355X (gfx950)", "buffer_bytes": 1 << 30,
                      "note": "factor = known bytes / counted bytes of one dispatch (multiply FETCH_SIZE or "
                              "WRITE_SIZE of a kernel with that access pattern by it)", "patterns": table}, indent=1))


if __name__ == "__main__":
    main()
