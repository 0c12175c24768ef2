"""HBM traffic per launch of the dominant kernel from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; separate passes, MI355X_MICROARCH.md §HBM):
    python tools/traffic.py <pmc1 counter_collection.csv> <pmc2 csv> <kernel substring> <out.json>
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes
of wide (16 B/lane) coalesced reads, so it is doubled (the guide's correction).
Dispatches are ranked by duration-independent size: the top half (the batch
launches, not the empty list-mode launches) is averaged."""
import csv, json, sys, statistics


def per_dispatch(path, counter, ksub):
    d = {}
    for r in csv.DictReader(open(path)):
        if ksub in r.get("Kernel_Name", "") and r["Counter_Name"] == counter:
            d[r.get("Dispatch_Id", r.get("Correlation_Id"))] = d.get(r.get("Dispatch_Id"), 0.0) + float(r["Counter_Value"])
    v = sorted(d.values())
    return v[len(v) // 2:] if v else []


def main():
    f1, f2, ksub, out = sys.argv[1:5]
    fetch = per_dispatch(f1, "FETCH_SIZE", ksub)
    write = per_dispatch(f2, "WRITE_SIZE", ksub)
    fb = statistics.mean(fetch) * 1024 * 2
    wb = statistics.mean(write) * 1024
    res = {"kernel": ksub, "hbm_bytes_per_launch": round(fb + wb), "fetch_bytes": round(fb), "write_bytes": round(wb),
           "dispatches": [len(fetch), len(write)],
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; KiB x1024; FETCH x2 (gfx950)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
