"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE; separate passes, MI355X_MICROARCH.md §HBM):
    python tools/traffic.py <pmc1 counter_collection.csv> <pmc2 csv> <kernel substring> <out.json>
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes
of wide (16 B/lane) coalesced reads, so it is doubled (the guide's correction).
Dispatches of the named (dominant) kernel are ranked by size and the top half
(the batch launches, not the empty list-mode launches) is averaged; every other
j2t/t2j/pack kernel of the same run is reported beside it the same way."""
import csv, json, sys, statistics, collections, re


def per_kernel(path, counter):
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r.get("Kernel_Name", "")
        m = re.search(r"(j2t_\w+|t2j_\w+|dg_pack\w*)", k)
        if not m:
            continue
        did = r.get("Dispatch_Id", r.get("Correlation_Id"))
        d[m.group(1)][did] = d[m.group(1)].get(did, 0.0) + float(r["Counter_Value"])
    return {k: sorted(v.values()) for k, v in d.items()}


def top_half_mean(v):
    """mean of the batch launches: dispatches at least half the largest
    (drops list-mode passes with nothing to do and single-message Do calls)"""
    if not v:
        return 0.0
    big = [x for x in v if x >= v[-1] / 2]
    return statistics.mean(big)


def exact_fetch(path):
    """kernel -> fetched bytes per dispatch from the L2's read requests by
    size (TCC_EA0_RDREQ_32B / _64B / _128B, one pass): 32 a + 64 b + 128 c.
    gfx950's FETCH_SIZE tallies 128-byte requests at 64 B (the guide's x2
    correction assumes every request is one); this is the count itself."""
    sizes = {"TCC_EA0_RDREQ_32B": 32, "TCC_EA0_RDREQ_64B": 64, "TCC_EA0_RDREQ_128B": 128}
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        c = r["Counter_Name"]
        if c not in sizes:
            continue
        m = re.search(r"(j2t_\w+|t2j_\w+|dg_pack\w*)", r.get("Kernel_Name", ""))
        if not m:
            continue
        did = r.get("Dispatch_Id", r.get("Correlation_Id"))
        d[m.group(1)][did] += float(r["Counter_Value"]) * sizes[c]
    return {k: sorted(v.values()) for k, v in d.items()}


def main():
    f1, f2, ksub, out = sys.argv[1:5]
    f3 = sys.argv[5] if len(sys.argv) > 5 else None  # optional: the request-size pass
    fetch, write = per_kernel(f1, "FETCH_SIZE"), per_kernel(f2, "WRITE_SIZE")
    exact = exact_fetch(f3) if f3 else {}
    kern = {}
    for k in sorted(set(fetch) | set(write)):
        fb = top_half_mean(fetch.get(k, [])) * 1024 * 2
        wb = top_half_mean(write.get(k, [])) * 1024
        kern[k] = {"hbm_bytes_per_launch": round(fb + wb), "fetch_bytes": round(fb), "write_bytes": round(wb),
                   "dispatches": [len(fetch.get(k, [])), len(write.get(k, []))]}
        if k in exact:
            fe = top_half_mean(exact[k])
            kern[k]["fetch_bytes_by_request_size"] = round(fe)
            kern[k]["hbm_bytes_per_launch_by_request_size"] = round(fe + wb)
    main_k = kern[ksub]
    res = {"kernel": ksub, **main_k, "all_kernels": kern,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; KiB x1024; FETCH x2 (gfx950); "
                     "per kernel: mean of its dispatches of at least half the largest one's size" +
                     ("; fetch_bytes_by_request_size: a third pass, TCC_EA0_RDREQ_32B/_64B/_128B x 32/64/128 B"
                      if f3 else "")}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
