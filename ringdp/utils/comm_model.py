"""Cost model of one bucket all-reduce, used to place bucket collectives in the captured step.

Where the numbers come from (all measured on MI355X by ``tools/comm_bench.py``; no multi-GPU box was
available to this work, so the N>1 terms are fitted on ranks SHARING one GPU and carry that caveat):

* latency term: the small-message floor of ringdp's xGMI all-reduce (the same IPC flag protocol as
  over real links) - 8.55 us at ws2 and 15.1 us at ws4 for 77 KB (``profiles/r05/xgmi/ws2_b128_s16.jsonl``,
  ``ws4_b128_s16.jsonl``).  A line through both: ``LAT0_US + LAT_RANK_US * (N - 1)`` = 5.3 + 3.25 (N - 1):
  28 us at N=8.  At N=1 (forced one-rank collectives) the collective is a local copy at ~1.5 TB/s (RCCL's
  one-rank floor is 3.1-4.0 us, ``profiles/comm_bench_r02_ws1.jsonl``, mostly launch cost that the graph
  hides).
* bandwidth term: a ring moves 2 (N-1)/N x S bytes per rank.  The shared-GPU sweeps give 391 GB/s (ws2)
  and 239 GB/s (ws4) bus bandwidth between 4 and 26 MB, but those are HBM-bound copies on one card; over
  real links one xGMI link is ~153 GB/s per direction.  ``RING_BW_GBPS`` = 100 takes one
  link at ~65 % efficiency: pessimistic for RCCL's multi-ring schedule over 7 links, so it over-estimates
  large buckets, which only makes the split placement below split MORE of them.
* one-shot (``RINGDP_P2P_ALLREDUCE_MAX_BYTES``, rccl_pg.cpp): every rank reads the N-1 peers' buckets
  directly, one peer per link, in one handshake: the ws2 floor plus S at one link's ``RING_BW_GBPS``.
* a segment boundary of the split capture plus its two cross-queue waits costs 15-45 us (one-rank kernel
  traces, ``profiles/r05/split/``); ``SPLIT_MIN_US`` = 30 is the middle: a bucket whose collective is
  modelled shorter than that is cheaper inline on the compute stream than split off.

How the N=8 ConvNet placement follows: at B=65536 the two buckets are 369 KB (fc1 + conv3) and 76 KB
(conv2 + conv1).  Modelled ring times at N=8: 34.5 and 29.4 us.  The first exceeds 30 us and is split off
(it overlaps the ~0.9 ms conv2/conv1 backward); the second is the last bucket and always inline, so the
modelled exposed communication is 29.4 us of a ~3.4 ms step (E(8) ~ 0.99).  At B <= 4096 the bench uses
one 455 KB bucket, which is inline: 36.0 us ring / 13.1 us one-shot exposed per ~80 us step at B=100
(E(8) ~ 0.69 / 0.86) - the number the first 8-GPU run has to confirm or reject.
"""
from __future__ import annotations

from typing import Dict, List

LAT0_US = 5.3          # latency floor at N=2 minus one rank's increment (fit, see above)
LAT_RANK_US = 3.25     # latency increment per extra rank (ws2 -> ws4 fit)
ONE_RANK_BW_GBPS = 1500.0
RING_BW_GBPS = 100.0
SPLIT_MIN_US = 30.0


def est_us(nbytes: int, world: int, algo: str = "ring") -> float:
    """Modelled device time of one all-reduce of ``nbytes`` over ``world`` ranks."""
    if world <= 1:
        return nbytes / (ONE_RANK_BW_GBPS * 1e3)
    if algo == "oneshot":
        return LAT0_US + LAT_RANK_US + nbytes / (RING_BW_GBPS * 1e3)
    return LAT0_US + LAT_RANK_US * (world - 1) + 2.0 * (world - 1) / world * nbytes / (RING_BW_GBPS * 1e3)


def exposed_us(plan: List[Dict], world: int, algo: str = "ring") -> float:
    """Modelled communication time NOT hidden behind backward, for a placement ``plan`` (the split
    capture's ``split_info``): inline collectives run on the compute stream and are fully exposed;
    split / deferred ones are taken as hidden (they run while the rest of backward runs)."""
    return sum(est_us(b["bytes"], world, algo) for b in plan
               if str(b.get("placement", "inline")).startswith("inline"))


def replan(plan: List[Dict], world: int, min_us: float = SPLIT_MIN_US) -> List[Dict]:
    """The placement the split capture (ringdp.utils.graph.StepGraph.capture_split) would choose for the
    same buckets at ``world`` ranks: split where the modelled collective is at least ``min_us`` (never the
    last bucket), deferred behind an earlier split, else inline."""
    out, split = [], False
    for i, b in enumerate(plan):
        if i == len(plan) - 1:
            pl = "inline (last)"
        elif est_us(b["bytes"], world) >= min_us:
            pl, split = "split", True
        else:
            pl = "deferred to the next boundary" if split else "inline"
        out.append(dict(b, placement=pl))
    return out


def scaling_model(plan: List[Dict], step_us: float, world_now: int, worlds=(2, 4, 8), split: bool = True) -> Dict:
    """Modelled exposed comm and weak-scaling efficiency at other world sizes, from this run's plan and
    step time.  The comm-free step time is the measured step minus this run's modelled inline comm.  With
    ``split`` (the captured step is segment-split), each world size gets its own placement (``replan``)."""
    base = max(step_us - exposed_us(plan, world_now), 1e-3)
    out: Dict = {"comm_free_step_us": round(base, 2), "assumptions": "ringdp.utils.comm_model (fitted on "
                 "ranks sharing one MI355X; no multi-GPU measurement behind the N>1 terms)"}
    for n in worlds:
        p = replan(plan, n) if split else plan
        ring = exposed_us(p, n, "ring")
        one = exposed_us(p, n, "oneshot")
        out[str(n)] = {"placement": [b["placement"] for b in p],
                       "exposed_us_ring": round(ring, 2), "exposed_us_oneshot": round(one, 2),
                       "E_ring": round(base / (base + ring), 3), "E_oneshot": round(base / (base + one), 3)}
    return out
