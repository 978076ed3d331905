"""HBM traffic per launch of the grouped dW kernel from the two rocprofv3 PMC passes that
tools/prof_round2.sh collects (FETCH_SIZE and WRITE_SIZE in separate runs), against the
kernel's algorithmic bytes; writes profiles/round2/pmc_traffic_<cfg>.json (read by bench.py).

    python tools/pmc_traffic.py gpurun_out/r2_c4 c4 <commit>

HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB units; gfx950 counts wide streaming reads at
half, MI355X_MICROARCH.md HBM/rocprofv3 section).  Algorithmic bytes of a launch = the dY and X
operands (bf16) once + dW (fp32) once for every block of its group."""
import csv
import glob
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from bench import CONFIGS  # noqa: E402

KERNEL = "gemm_dw_kernel"


def launches(d, counter):
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]) * 1024))
    rows.sort()
    return rows


def block_bytes(c):
    d, L = c["n_embd"], c["n_layer"]
    hd = d // c["n_head"]
    kvd = (c["kv"] or c["n_head"]) * hd
    nqkv = d + 2 * kvd
    M = c["batch"] * c["block_size"]
    if c["swiglu"]:
        hp = -(-int(8 * d // 3) // 64) * 64
        prods = [(d, hp), (2 * hp, d), (d, d), (nqkv, d)]
    else:
        prods = [(d, 4 * d), (4 * d, d), (d, d), (nqkv, d)]
    return sum(2 * M * (n + k) + 4 * n * k for n, k in prods), sum(4 * n * k for n, k in prods)


def main():
    d, cfg, commit = sys.argv[1], sys.argv[2], sys.argv[3]
    c = CONFIGS[cfg]
    fetch, write = launches(f"{d}/pmc_fetch", "FETCH_SIZE"), launches(f"{d}/pmc_write", "WRITE_SIZE")
    assert fetch and len(fetch) == len(write), (len(fetch), len(write))
    per_block, dw_block = block_bytes(c)
    out = []
    for (_, name, fb), (_, _, wb) in zip(fetch, write):
        # the launch writes its blocks' fp32 dW once: WRITE_SIZE / dW bytes per block = group size
        blocks = max(1, round(wb / dw_block))
        out.append({"kernel": name, "blocks": blocks, "fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": 2 * fb + wb,
                    "algorithmic_bytes": blocks * per_block})
    res = {"probe": "gemm_dw_grouped", "kernel": sorted({o["kernel"] for o in out}), "config": cfg, "commit": commit,
           "hbm_bytes_per_launch": round(sum(o["hbm_bytes"] for o in out) / len(out)),
           "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of `python "
                     "bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-kernel-roofline`; HBM bytes = 2 x "
                     "FETCH_SIZE (gfx950 counts wide streaming reads at half) + WRITE_SIZE, KB units; algorithmic = "
                     "dY and X operands (bf16) once + dW (fp32) once per block in the group",
           "launches": out}
    res["algorithmic_bytes_per_launch"] = round(sum(o["algorithmic_bytes"] for o in out) / len(out))
    res["ratio"] = round(res["hbm_bytes_per_launch"] / res["algorithmic_bytes_per_launch"], 3)
    dst = ROOT / "profiles" / "round2" / f"pmc_traffic_{cfg}.json"
    dst.write_text(json.dumps(res, indent=1) + "\n")
    print(dst, res["hbm_bytes_per_launch"], res.get("ratio"))


if __name__ == "__main__":
    main()
