#!/usr/bin/env python3
"""profiles/traffic.json entries from one HEAD measurement (tools/gpu_measure.sh
-> pmc.json, summarised by tools/pmc_parse.py), so every `traffic` / request /
instruction figure in bench.py's line comes from the same dated file.

usage: pmc_to_traffic.py PMC.json SOURCE-LABEL [workload=c3] [out=profiles/traffic.json]

Per kernel, per launch (the steady launches' mean):
  * HBM traffic: FETCH_SIZE (KiB) x 2 + WRITE_SIZE (KiB), the guide's gfx950
    read correction (MI355X_MICROARCH.md: FETCH_SIZE = TCC_EA0_RDREQ x 64 B
    and reads half the bytes of a wide streaming read), both raw counters kept;
  * the L2: TCC_HIT / TCC_MISS and the memory-side reads TCC_EA0_RDREQ;
  * the TCP->TCC requests (read / write / atomic);
  * SQ instruction counts (VALU / SALU / VMEM / LDS).
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = ("profiles/r01_probe_random_access.jsonl: random 8-B loads over a 2 GB table, 54.1 G/s (200 MB: 55.7 G/s; "
         "L2-resident 4 MB: 251 G/s)")


def find(pmc, prefix):
    for k, v in pmc.items():
        if k.startswith(prefix) or k.startswith("gsim::" + prefix):
            return k, v
    raise SystemExit(f"no kernel {prefix} in the counters")


def traffic(v):
    f, w = v["FETCH_SIZE"], v["WRITE_SIZE"]
    return {"bytes_per_launch": (2 * f + w) * 1024, "bytes_per_launch_raw": (f + w) * 1024,
            "fetch_kib_raw": f, "write_kib_raw": w}


def l2(v):
    hit, miss = v["TCC_HIT_sum"], v["TCC_MISS_sum"]
    return {"tcc_hit": hit, "tcc_miss": miss, "hit_rate": hit / max(1.0, hit + miss),
            "tcc_ea0_rdreq": v["TCC_EA0_RDREQ_sum"]}


def reqs(v):
    r, w = v["TCP_TCC_READ_REQ_sum"], v["TCP_TCC_WRITE_REQ_sum"]
    a1, a0 = v["TCP_TCC_ATOMIC_WITH_RET_REQ_sum"], v["TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum"]
    return {"requests_per_launch": r + w + a1 + a0, "read": r, "write": w, "atomic_with_ret": a1,
            "atomic_without_ret": a0}


def sq(v):
    return {c.lower(): v[c] for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                                      "SQ_INSTS_LDS", "SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY") if c in v}


def main():
    pmc = json.load(open(sys.argv[1]))
    src = sys.argv[2]
    wl = sys.argv[3] if len(sys.argv) > 3 else "c3"
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(REPO, "profiles", "traffic.json")
    data = json.load(open(out)) if os.path.exists(out) else {}
    corr = "read side x2 (gfx950 FETCH_SIZE under-count, MI355X_MICROARCH.md), write exact"
    kr, vr = find(pmc, "k_refresh_score<true, true>")
    data[wl] = dict(traffic(vr), **l2(vr), kernel=kr, launches=vr["_launches"], correction=corr, source=src)
    ks, vs = find(pmc, "k_send_tm<")
    kc, vc = find(pmc, "k_commit<")
    ts, tc = traffic(vs), traffic(vc)
    data[wl + ":send"] = dict(
        bytes_per_launch=ts["bytes_per_launch"] + tc["bytes_per_launch"],
        bytes_per_launch_raw=ts["bytes_per_launch_raw"] + tc["bytes_per_launch_raw"],
        per_kernel={ks: dict(ts, **l2(vs)), kc: dict(tc, **l2(vc))},
        kernel=f"{ks} + {kc} (one launch each per propagation round)", correction=corr,
        calibration=("k_send_tm's accesses are 1-8 B gathers and atomics at random addresses: a miss moves a "
                     "whole line, and the x2 read correction is calibrated for 16-B/lane streaming reads only; "
                     "bytes_per_launch_raw is the uncorrected count"),
        source=src)
    data[wl + ":send_req"] = dict(reqs(vs), **l2(vs), kernel=ks, ceiling_req_per_s=54e9, ceiling_source=PROBE,
                                  commit=dict(reqs(vc), **l2(vc), kernel=kc), source=src)
    kh, vh = find(pmc, "k_heartbeat<32>")
    data[wl + ":hb_valu"] = dict(valu_insts_per_launch=vh["SQ_INSTS_VALU"], salu_insts_per_launch=vh["SQ_INSTS_SALU"],
                                 waves_per_launch=vh["SQ_WAVES"], peak_wave_insts_per_s=256 * 4 * 2.4e9 / 2,
                                 peak_source=("MI355X_MICROARCH.md: 256 CUs x 4 SIMDs x 2.4 GHz, a wave64 VALU op "
                                              "issues over 2 cycles"),
                                 sq=sq(vh), traffic=traffic(vh), l2=l2(vh), kernel=kh, source=src)
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps({k: data[k].get("bytes_per_launch", data[k].get("requests_per_launch")) for k in data}))


if __name__ == "__main__":
    main()
