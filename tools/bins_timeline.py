#!/usr/bin/env python3
"""Analyses the per-item records of k_render_bins written by a
BIH_BINS_TIMELINE=1 build (bih_sync appends one block per synchronised call
to $BIH_TIMELINE_OUT; tools/call_breakdown.py --sync 1 makes one block per
launch).  Per launch: span (first wave start -> last wave exit), items, item
durations, when the queue ran dry (last item start) and the tail after it,
wave-slot utilisation (item time / (waves x span)) and its profile over the
span in tenths.  Times: s_memrealtime, 100 MHz (10 ns).
usage: tools/bins_timeline.py FILE [--skip N] [--show K]"""
import argparse
import struct

import numpy as np


def blocks(path):
    data = open(path, "rb").read()
    off = 0
    while off + 16 <= len(data):
        magic, n, lost, _ = struct.unpack_from("<4I", data, off)
        if lost:
            print(f"(block with {lost} records dropped: more items per wave than the buffer holds)")
        off += 16
        if magic != 0x544C4942:
            raise SystemExit("bad block header")
        rec = np.frombuffer(data, dtype=np.uint32, count=4 * n, offset=off).reshape(n, 4).astype(np.int64)
        off += 16 * n
        yield rec


def analyse(rec):
    # kind 4 (item counters) follows its live item (kind 0) in the wave's run:
    # pair them, then drop them from the time records
    kind_all = rec[:, 0] >> 28
    stats = {}
    if (kind_all == 4).any():
        idx4 = np.nonzero(kind_all == 4)[0]
        prev = idx4 - 1
        ok = (prev >= 0) & (kind_all[np.maximum(prev, 0)] == 0)
        for i4, p in zip(idx4[ok], prev[ok]):
            ent, mt = int(rec[i4, 1]), int(rec[i4, 2])
            stats[int(p)] = (ent, mt, int(rec[i4, 3] & 0xFFFF), int(rec[i4, 3] >> 16))
        keep = kind_all != 4
        remap = np.cumsum(keep) - 1
        stats = {int(remap[k]): v for k, v in stats.items()}
        rec = rec[keep]
    wave = rec[:, 0] & 0xFFFFFF
    xcc = (rec[:, 0] >> 24) & 15
    kind = rec[:, 0] >> 28
    t = rec[:, 1].copy()
    t = (t - t[0] + (1 << 31)) % (1 << 32) - (1 << 31)    # unwrap relative to the first record
    t -= t.min()
    dur = rec[:, 2]
    ln = rec[:, 3] & 0xFFFFFF             # live items: list length | frames << 24
    frames = rec[:, 3] >> 24
    starts, exits = t[kind == 2], t[kind == 3]
    span = (exits.max() - starts.min()) / 100.0          # us
    items = kind <= 1
    live, bg = kind == 0, kind == 1
    it_s, it_e = t[items] / 100.0, (t[items] + dur[items]) / 100.0
    nwaves = int((kind == 2).sum())
    last_start = it_s.max()
    busy = dur[items].sum() / 100.0
    prof = []
    edges = np.linspace(0, span, 11)
    for a, b in zip(edges[:-1], edges[1:]):
        ov = np.clip(np.minimum(it_e, b) - np.maximum(it_s, a), 0, None).sum()
        prof.append(ov / (nwaves * (b - a)))
    d_live = dur[live] / 100.0
    q = lambda v, f: float(np.quantile(v, f)) if v.size else 0.0
    # per wave: its start (kind 2) and its first item's start (the queue's
    # start-up cost), its last item's end and its exit
    first_item, wstart = {}, {}
    for w_, k_, t_ in zip(wave.tolist(), kind.tolist(), t.tolist()):
        if k_ == 2:
            wstart[w_] = t_
        elif k_ <= 1 and w_ not in first_item:
            first_item[w_] = t_
    gaps = np.array([first_item[w_] - wstart[w_] for w_ in first_item if w_ in wstart]) / 100.0
    ws = np.array(list(wstart.values())) / 100.0
    out = {
        "span_us": span, "waves": nwaves,
        "wave_start_us_q50_q90_max": [float(np.quantile(ws, .5)), float(np.quantile(ws, .9)), float(ws.max())]
        if ws.size else None,
        "start_to_first_item_us_q10_q50_q90": [float(np.quantile(gaps, f)) for f in (.1, .5, .9)] if gaps.size else None, "items_live": int(live.sum()), "items_bg": int(bg.sum()),
        "utilisation": busy / (nwaves * span),
        "queue_dry_us": float(last_start), "tail_us": span - float(last_start),
        "wave_exit_q10_q50_q90_us": [q(exits / 100.0, 0.1), q(exits / 100.0, 0.5), q(exits / 100.0, 0.9)],
        "live_item_us_mean_p50_p90_p99_max": [float(d_live.mean()) if d_live.size else 0.0, q(d_live, .5),
                                             q(d_live, .9), q(d_live, .99), float(d_live.max()) if d_live.size else 0.0],
        "bg_item_us_mean": float((dur[bg] / 100.0).mean()) if bg.any() else 0.0,
        "profile_tenths": [round(x, 3) for x in prof],
        "xcd_exit_us": [round(float(exits[xcc[kind == 3] == x].max() / 100.0), 1) if (xcc[kind == 3] == x).any()
                        else None for x in range(8)],
    }
    # the longest live items: start, duration, list length
    if live.any():
        idx = np.argsort(-dur[live])[:5]
        ls, ld, ll, lf = t[live][idx] / 100.0, dur[live][idx] / 100.0, ln[live][idx], frames[live][idx]
        out["longest_live (start us, us, list length, frames)"] = [
            (round(float(a), 1), round(float(b), 1), int(c), int(f)) for a, b, c, f in zip(ls, ld, ll, lf)]
        out["live_items_by_frames"] = {int(f): int((frames[live] == f).sum()) for f in np.unique(frames[live])}
        if stats:
            li = np.nonzero(live)[0]
            order = li[np.argsort(-dur[li])]
            rows = []
            for k in order[:8]:
                e, m, pv, pl = stats.get(int(k), (0, 0, 0, 0))
                f = max(1, int(frames[k]))
                rows.append((round(float(dur[k]) / 100.0 / f, 1), int(ln[k]), round(e / f, 1), round(m / f, 1),
                             round(pv / f, 1), round(pl / f, 1)))
            out["longest per frame (us, list, entries, mt, path-table lanes, plan lanes)"] = rows
            # correlation of per-frame duration with each counter
            d = np.array([dur[k] / 100.0 / max(1, frames[k]) for k in li if int(k) in stats])
            cs = np.array([stats[int(k)] for k in li if int(k) in stats], dtype=float)
            fr = np.array([max(1, frames[k]) for k in li if int(k) in stats], dtype=float)[:, None]
            cs = cs / fr
            if d.size > 10:
                out["corr(us/frame; entries, mt, path, plan)"] = [round(float(np.corrcoef(d, cs[:, j])[0, 1]), 3)
                                                                 for j in range(4)]
                top = d >= np.quantile(d, 0.99)
                out["mean per frame, top 1% vs all (entries, mt, path, plan)"] = [
                    [round(float(x), 1) for x in cs[top].mean(0)], [round(float(x), 1) for x in cs.mean(0)]]
        # items that end in the last 10 % of the span
        late = (it_e > 0.9 * span) & (kind[items] == 0)
        out["live_items_ending_in_last_tenth"] = int(late.sum())
        # list length vs duration (mean per list-length class)
        cls = np.floor(np.log2(np.maximum(ln[live], 1))).astype(int)
        out["us_by_log2_list_len"] = {int(c): (int((cls == c).sum()), round(float(d_live[cls == c].mean()), 2))
                                      for c in np.unique(cls)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("file")
    ap.add_argument("--skip", type=int, default=2, help="blocks to skip (warm-up)")
    ap.add_argument("--show", type=int, default=3)
    a = ap.parse_args()
    res = [analyse(r) for r in blocks(a.file)][a.skip:]
    for r in res[:a.show]:
        print("---")
        for k, v in r.items():
            print(f"  {k}: {v}")
    if res:
        keys = ["span_us", "utilisation", "queue_dry_us", "tail_us"]
        print("mean over %d launches:" % len(res), {k: round(float(np.mean([r[k] for r in res])), 3) for k in keys})
        print("mean profile:", [round(float(x), 3) for x in np.mean([r["profile_tenths"] for r in res], 0)])


if __name__ == "__main__":
    main()
