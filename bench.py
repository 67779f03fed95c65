#!/usr/bin/env python3
"""Self-play throughput bench (BASELINE.json metric: MCTS node-expansions/s/GPU @400 sims;
self-play games/s at 1/2/4/8 GPUs).

One "step" = one self-play ply in every game slot = `games` searches of `sims` simulations
(select -> fused ResNet leaf evaluation -> expand/backup, each simulation one NN evaluation,
SURVEY.md 8d) + the move/record/deal kernel. Inputs (decks, trees, weights) are resident in
HBM before the timed region. Multi-GPU: one process per GPU (torchrun), games sharded by
global game id, no collective inside the timed region; the (s, pi, z) all-gather over RCCL
runs after it and is reported separately.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5]
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "onitama-alphazero_amd"))

import torch  # noqa: E402  (imported before the engine so both share one HIP runtime)
import torch.distributed as dist  # noqa: E402

CONFIGS = {
    # BASELINE.json configs[1]: 4096 parallel games, 100 sims/move, 3-block fp32, 1 GPU
    "c2": dict(games=4096, sims=100, blocks=3, fixed_deck=1, precision="fp32"),
    # configs[2]: 65536 parallel games, 400 sims/move, 1 GPU (the metric's "@400 sims"); fp32 NN
    # arithmetic (north star: policy/value within 1e-4 fp32) on the fp16x3 split kernel by default
    "c3": dict(games=65536, sims=400, blocks=3, fixed_deck=1, precision="fp32"),
    # configs[4] (per GPU): 16-card random deals, 800 sims, 6-block, bf16 MFMA inputs / fp32 accumulate
    "c5": dict(games=65536, sims=800, blocks=6, fixed_deck=0, precision="bf16"),
}
FLOP_PER_SIM = {3: 11_681_928, 5: 19_054_728, 6: 22_741_128}  # dense MACs x 2


def nonzero_flop_per_sim(blocks):
    """FLOPs excluding products with the 3x3 convs' zero padding: 169 on-board (square, tap)
    pairs of 225 (what k_nn_sq16 executes)."""
    macs = 169 * 21 * 64 + blocks * 2 * 169 * 64 * 64 + (1600 + 1600 + 64 + 3200 + 2500)
    return 2 * macs
PEAK_TFLOPS = {"fp32": 157.3, "bf16": 2500.0}  # MI355X_MICROARCH.md: F32 matrix / BF16 dense MFMA peaks (spec)
# fp32 split kernel (OAZ_FP32_SPLIT): every fp32 MAC is six bf16 MFMA products, so its MFMA ceiling
# in fp32 FLOP/s is the bf16 dense peak / 6
PEAK_TFLOPS["fp32_split"] = PEAK_TFLOPS["bf16"] / 6.0
# fp16 split kernel (OAZ_FP32_SPLIT16): three fp16 MFMA products per fp32 MAC (fp16 and bf16 MFMA
# share one rate on gfx950), so its ceiling is the dense fp16 peak / 3
PEAK_TFLOPS["fp32_split16"] = PEAK_TFLOPS["bf16"] / 3.0
NN_KERNEL = {"fp32": "k_nn_sq16<fp32> (fused ResNet, exact fp32 v_mfma_f32_16x16x4_f32)",
             "fp32_split": "k_nn_x6 (fused ResNet, fp32 operands split exactly into 3 bf16 terms, 6 products on "
                           "v_mfma_f32_16x16x32_bf16, fp32 accumulate)",
             "fp32_split16": "k_nn_h3 (fused ResNet, fp32 operands split into hi+lo fp16 terms, 3 products on "
                             "v_mfma_f32_16x16x32_f16, fp32 accumulate)",
             "bf16": "k_nn_h3 in bf16 mode (fused ResNet, transposed tiles, one bf16 product on "
                     "v_mfma_f32_16x16x32_bf16, fp32 accumulate)"}
METRIC = "MCTS node-expansions/sec/GPU @400 sims; self-play games/sec at 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=14)
    ap.add_argument("--stagger", type=int, default=12,
                    help="slot g starts after g %% stagger plies so game ages reach steady state in warmup")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--games", type=int, default=0, help="override games per GPU")
    ap.add_argument("--sims", type=int, default=0, help="override sims per move")
    ap.add_argument("--fp32-kernel", default="split16", choices=["split", "split16", "exact"],
                    help="fp32 NN kernel: split (bf16x6), split16 (fp16x3; both fp32-level error) or exact "
                         "(fp32 MFMA products)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="cpu_baseline sample length")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--no-exact", action="store_true", help="skip the exact-fp32 comparison leg")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 FETCH/WRITE_SIZE child passes")
    ap.add_argument("--no-noise", action="store_true", help=argparse.SUPPRESS)  # experiments only: not C3
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-plies", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--pmc-parts", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--mode", default="selfplay", choices=["selfplay", "train", "pure_mcts", "arena"],
                    help="train: SGD steps of the training loop (SURVEY 8f #2), not the headline metric")
    ap.add_argument("--train-blocks", type=int, default=5, help="train mode: residual blocks (bin/train.rs:60)")
    ap.add_argument("--pm-games", type=int, default=1048576,
                    help="pure_mcts mode: searches per launch (1 M: 933 M playouts/s vs 695 M at 256 k, the "
                         "divergent rollouts' tail amortised over two rounds of waves; 2 M: 319 M, 134 GB of trees "
                         "past the TLB's reach; DESIGN.md section 8)")
    ap.add_argument("--arena-games", type=int, default=131072,
                    help="arena mode: games per fight per GPU (a fight lasts as long as its longest game, so small "
                         "fights are tail-bound: 65 536 games 4 338 games/s, 131 072 5 112; two engines of ~70 GB)")
    ap.add_argument("--pm-playouts", type=int, default=400, help="pure_mcts mode: playouts per search")
    ap.add_argument("--train-batch", type=int, default=512, help="train mode: global batch (train.rs:142)")
    return ap.parse_args()


def pmc_traffic(args, cfg):
    """HBM bytes per launch of k_nn_h3 and the tree kernels from rocprofv3 PMC counters, one counter
    per pass (TCC slots: FETCH_SIZE and WRITE_SIZE do not fit one pass). Each pass profiles a child
    that plays the bench's warm-up plies (same stagger, full sims) unprofiled and collects counters
    only on the simulation steps of the NEXT ply (--kernel-iteration-range, per kernel), so the
    tree kernels are measured on steady-state trees, as timed. Runs as child processes BEFORE this
    process touches the GPU. gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half
    the bytes of wide (16 B/lane) coalesced reads -> doubled; WRITE_SIZE is taken as reported."""
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    parts = sim_parts(cfg["games"])  # launches of each kernel per simulation step
    # the profiled ply follows the bench's warm-up plies, but its first kernel index stays at most
    # ~11 200 (C5's 14 x 1 600 launches made the rocprofv3 counter child crash on the host): where the
    # game parts would push it past that, the child runs one part (half the launches per ply, the same
    # positions and trees per simulation step), so C5 is also profiled after all 14 warm-up plies
    if args.warmup * cfg["sims"] * parts > 11200:
        parts = 1
    per_ply = cfg["sims"] * parts
    plies = min(args.warmup, max(1, 11200 // per_ply))
    # with fewer warm-up plies than the timed region follows, the staggered starts are compressed to
    # them (every slot playing, game ages spread over `plies` plies) so the profiled ply is steady state
    stagger = min(args.stagger, plies) if args.stagger > 1 else 0
    first, last = plies * per_ply + 1, (plies + 1) * per_ply  # 1-based launch index of each kernel
    kb, tree_kb, counts = {}, {"backup_select": {}}, {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        with tempfile.TemporaryDirectory() as d:
            cmd = [prof, "--pmc", ctr, "--kernel-include-regex", "k_nn_|k_backup_select",
                   "--kernel-iteration-range", f"[{first}-{last}]", "--output-format", "csv", "-d", d, "-o", "pmc",
                   "--", sys.executable, str(Path(__file__).resolve()), "--pmc-child", "--pmc-plies", str(plies),
                   "--stagger", str(stagger), "--warmup", str(plies), "--config", args.config, "--games", str(cfg["games"]),
                   "--sims", str(cfg["sims"]), "--fp32-kernel", args.fp32_kernel, "--pmc-parts", str(parts)]
            try:
                subprocess.run(cmd, timeout=600, capture_output=True, check=True)
            except (subprocess.SubprocessError, OSError) as exc:
                tail = getattr(exc, "stderr", None) or b""
                tail = tail.decode(errors="replace") if isinstance(tail, bytes) else str(tail)
                print(f"bench: PMC pass {ctr} failed ({type(exc).__name__}); child stderr:\n{tail[-6000:]}",
                      file=sys.stderr)
                return None
            rows = {"nn": [], "backup_select": []}
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if r["Counter_Name"] != ctr:
                        continue
                    k = ("nn" if "k_nn_" in r["Kernel_Name"] else "backup_select" if "k_backup_select" in r["Kernel_Name"]
                         else None)
                    if k:
                        rows[k].append((int(r.get("Dispatch_Id", 0) or 0), float(r["Counter_Value"])))
            if not rows["nn"]:  # C2: the one-launch-per-chunk kernel k_search_grp runs the whole search
                return pmc_grp_traffic(args, cfg, plies, stagger)
            for k, v in rows.items():  # the last ply's launches only (also if the range was not applied)
                v.sort()
                rows[k] = [x for _, x in v[-per_ply:]]
                counts[k] = len(rows[k])
            kb[ctr] = sum(rows["nn"]) / len(rows["nn"])
            for k in ("backup_select",):
                if rows[k]:
                    tree_kb[k][ctr] = sum(rows[k]) / len(rows[k])
    # the tree kernel's VALU work (one more pass, SQ block): instructions per wave and per simulation
    sq = {}
    with tempfile.TemporaryDirectory() as d:
        cmd = [prof, "--pmc", "SQ_INSTS_VALU", "SQ_WAVES", "--kernel-include-regex", "k_backup_select",
               "--kernel-iteration-range", f"[{first}-{last}]", "--output-format", "csv", "-d", d, "-o", "pmc",
               "--", sys.executable, str(Path(__file__).resolve()), "--pmc-child", "--pmc-plies", str(plies),
               "--stagger", str(stagger), "--warmup", str(plies), "--config", args.config, "--games", str(cfg["games"]),
               "--sims", str(cfg["sims"]), "--fp32-kernel", args.fp32_kernel, "--pmc-parts", str(parts)]
        try:
            subprocess.run(cmd, timeout=600, capture_output=True, check=True)
            per = {}
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if "k_backup_select" in r["Kernel_Name"]:
                        key = (int(r.get("Dispatch_Id", 0) or 0), r["Counter_Name"])
                        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
            ids = sorted({i for i, _ in per})[-per_ply:]
            valu = [per.get((i, "SQ_INSTS_VALU"), 0.0) for i in ids]
            waves = [per.get((i, "SQ_WAVES"), 0.0) for i in ids]
            if ids and sum(waves) > 0:
                games_per_launch = cfg["games"] / parts
                sq = {"valu_instructions_per_wave": sum(valu) / sum(waves),
                      "valu_instructions_per_sim": sum(valu) / len(ids) / games_per_launch,
                      "valu_cycles_per_simd_per_launch": VALU_CYC * sum(valu) / len(ids) / SIMDS,
                      "launches": len(ids)}
        except (subprocess.SubprocessError, OSError) as exc:
            print(f"bench: PMC pass SQ_INSTS_VALU failed ({type(exc).__name__})", file=sys.stderr)
    # per simulation step: its parts' launches
    fetch, write = 2.0 * kb["FETCH_SIZE"] * 1024.0 * parts, kb["WRITE_SIZE"] * 1024.0 * parts
    tree = {}
    for k, v in tree_kb.items():  # per game: a launch covers the game slots of one part
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            tree[k] = {"fetch_bytes_per_sim": 2.0 * v["FETCH_SIZE"] * 1024.0 * parts / cfg["games"],
                       "fetch_bytes_per_sim_raw": v["FETCH_SIZE"] * 1024.0 * parts / cfg["games"],
                       "write_bytes_per_sim": v["WRITE_SIZE"] * 1024.0 * parts / cfg["games"]}
    if sq and "backup_select" in tree:
        tree["backup_select"]["sq"] = sq
    return {"bytes_per_sim_step": fetch + write, "fetch_bytes": fetch, "write_bytes": write, "game_parts": parts,
            "raw_kb": kb, "tree_pmc": tree, "launches_profiled": counts,
            "note": f"rocprofv3 --pmc, separate passes, on the {cfg['sims']} simulation steps of ply {plies + 1} "
                    f"(after {plies} warm-up plies, stagger {stagger}); FETCH_SIZE x2 (gfx950 wide-read "
                    "correction)"}


def grp_launches_per_ply(sims):
    """k_search_grp launches per ply: one per root-noise chunk of max(16, min(512, sims)) simulations
    (oaz_engine.cpp noise_chunk_for; the engine is created with `sims`), i.e. a C2 ply is one launch."""
    c = max(16, min(512, sims))
    return (sims + c - 1) // c


def pmc_grp_traffic(args, cfg, plies, stagger):
    """The k_search_grp launches' HBM bytes (C2: up to 16 x CU-count games, one launch per noise chunk runs the
    walks, k_nn_h3's body and the backups of every game): FETCH_SIZE / WRITE_SIZE passes over the launches of
    the ply after `plies` warm-up plies, as pmc_traffic does for k_nn_h3."""
    prof = shutil.which("rocprofv3")
    per_ply = grp_launches_per_ply(cfg["sims"])  # k_search_grp launches per ply
    first, last = plies * per_ply + 1, (plies + 1) * per_ply
    kb = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        with tempfile.TemporaryDirectory() as d:
            cmd = [prof, "--pmc", ctr, "--kernel-include-regex", "k_search_grp",
                   "--kernel-iteration-range", f"[{first}-{last}]", "--output-format", "csv", "-d", d, "-o", "pmc",
                   "--", sys.executable, str(Path(__file__).resolve()), "--pmc-child", "--pmc-plies", str(plies),
                   "--stagger", str(stagger), "--warmup", str(plies), "--config", args.config, "--games", str(cfg["games"]),
                   "--sims", str(cfg["sims"]), "--fp32-kernel", args.fp32_kernel, "--pmc-parts", "1"]
            try:
                subprocess.run(cmd, timeout=600, capture_output=True, check=True)
            except (subprocess.SubprocessError, OSError) as exc:
                print(f"bench: PMC pass {ctr} (k_search_grp) failed ({type(exc).__name__})", file=sys.stderr)
                return None
            v = []
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if r["Counter_Name"] == ctr and "k_search_grp" in r["Kernel_Name"]:
                        v.append((int(r.get("Dispatch_Id", 0) or 0), float(r["Counter_Value"])))
            if not v:
                print(f"bench: PMC pass {ctr} collected no k_nn_ or k_search_grp rows", file=sys.stderr)
                return None
            v.sort()
            v = [x for _, x in v[-per_ply:]]
            kb[ctr] = sum(v) / len(v)
    fetch, write = 2.0 * kb["FETCH_SIZE"] * 1024.0, kb["WRITE_SIZE"] * 1024.0
    sims_per_launch = cfg["games"] * cfg["sims"] / per_ply
    return {"kernel": "k_search_grp", "bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
            "bytes_per_launch_raw": fetch / 2.0 + write,  # FETCH_SIZE x1: exact for scattered records
            "bytes_per_sim": (fetch + write) / sims_per_launch, "raw_kb": kb, "launches_profiled": per_ply,
            "note": f"rocprofv3 --pmc, separate passes, on the {per_ply} k_search_grp launches of ply {plies + 1} "
                    f"(after {plies} warm-up plies, stagger {stagger}); FETCH_SIZE x2 (gfx950 wide-read correction)"}


def pmc_clock(args, cfg):
    """The clock the NN kernel runs at, and its rocprofv3 kernel-trace duration on this box: one child
    pass `rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace` over the k_nn_ launches of one ply on ONE
    stream (oaz_config.parts = 1, the single-stream leg's shape) after 2 unprofiled warm-up plies.
    GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md 'DVFS give-back'): cycles per launch
    = GRBM_GUI_ACTIVE / 8, clock of a profiled launch = cycles / its traced duration. Cycles barely
    depend on the clock for an MFMA-bound kernel, so cycles / the un-profiled HIP-event launch time of
    the single-stream leg is the clock of the measured launches (bench main). Runs before this
    process touches the GPU."""
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    per_ply, plies = cfg["sims"], 2
    first, last = plies * per_ply + 1, (plies + 1) * per_ply
    with tempfile.TemporaryDirectory() as d:
        cmd = [prof, "--pmc", "GRBM_GUI_ACTIVE", "--kernel-trace", "--kernel-include-regex", "k_nn_",
               "--kernel-iteration-range", f"[{first}-{last}]", "--output-format", "csv", "-d", d, "-o", "clk",
               "--", sys.executable, str(Path(__file__).resolve()), "--pmc-child", "--pmc-plies", str(plies),
               "--pmc-parts", "1", "--stagger", "0", "--warmup", str(plies), "--config", args.config, "--games",
               str(cfg["games"]), "--sims", str(cfg["sims"]), "--fp32-kernel", args.fp32_kernel]
        try:
            subprocess.run(cmd, timeout=600, capture_output=True, check=True)
        except (subprocess.SubprocessError, OSError) as exc:
            tail = getattr(exc, "stderr", None) or b""
            tail = tail.decode(errors="replace") if isinstance(tail, bytes) else str(tail)
            print(f"bench: PMC clock pass failed ({type(exc).__name__}); child stderr:\n{tail[-4000:]}",
                  file=sys.stderr)
            return None
        grbm, dur = {}, {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and "k_nn_" in r["Kernel_Name"]:
                    grbm[int(r["Dispatch_Id"])] = grbm.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_nn_" in r["Kernel_Name"]:
                    dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    ids = sorted(set(grbm) & set(dur))[-per_ply:]
    if not ids:
        print("bench: PMC clock pass collected no k_nn_ rows", file=sys.stderr)
        return None
    cyc = sorted(grbm[i] / 8.0 for i in ids)
    clk = sorted(grbm[i] / 8.0 / dur[i] / 1e6 for i in ids if dur[i] > 0)
    ms = [dur[i] * 1e3 for i in ids]
    return {"cycles_per_launch": cyc[len(cyc) // 2], "profiled_clock_mhz": clk[len(clk) // 2],
            "profiled_avg_launch_ms": sum(ms) / len(ms), "launches": len(ids),
            "note": f"rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace, one stream, the {len(ids)} k_nn_ launches of "
                    f"ply {plies + 1} (median per launch; GRBM_GUI_ACTIVE / 8 XCDs = cycles)"}


HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E ~8 TB/s
SIMDS = 1024  # 256 CUs x 4 SIMDs
VALU_CYC = 2  # issue throughput of a wave64 32-bit VALU instruction on a SIMD-32 (MI355X_MICROARCH.md; f64 ops take more)
NOMINAL_MHZ = 2400.0  # MI355X_MICROARCH.md: max engine clock (the MFMA peaks are quoted at it)
XCDS = 8  # MI355X: 8 XCDs, each with its own L2 (written back and invalidated at kernel boundaries)
XGMI_LINK_GBPS = 153.0  # per direction per link (7 links per GPU), the all-gather's reference rate


class _StdoutToStderr:
    """fd-level redirect of stdout to stderr: RCCL prints its version banner to stdout while a
    communicator initialises, and the bench's stdout must stay ONE JSON line."""

    def __enter__(self):
        import ctypes
        sys.stdout.flush()
        self._libc = ctypes.CDLL(None)
        self._libc.fflush(None)
        self._saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        self._libc.fflush(None)
        os.dup2(self._saved, 1)
        os.close(self._saved)
        return False


def tree_roofline(kt, sims, sim_steps, expansions, depth, branching, cfg, pmc=None):
    """Achieved HBM-side bytes of the tree kernels (tree-kernel GB/s vs HBM peak),
    from the run's mean walk depth D and branching K and the 32-byte node layout:
    select reads the root state (24 B) and node (32 B), per level K children (32 B each), sqrt(N)
    (8 B) and writes a path entry (4 B), at the root K noise pairs (8 B each, training noise), and
    writes the leaf record (24 + 8 B) and two counters (16 B); expand/backup reads the leaf record
    and node (64 B) and the value (4 B), on expansion the policy row (200 B) and writes K fresh
    children (32 B each) and the header (16 B), and per path node reads the path entry (4 B) and
    updates N and W (12 B read + 12 B written)."""
    if not kt.backup_select_n:
        return None
    D, K = depth, branching
    per_launch = sims / max(1, sim_steps) / max(1, kt.parts)  # games per tree-kernel launch (one game part)
    noise = 8.0 * K if cfg.get("noise", True) else 0.0
    sel = 24 + 32 + D * (32 * K + 8 + 4) + noise + 32 + 16 + 1  # + the need flag
    exp = 64 + 4 + 4 + (expansions / max(1, sims)) * (200 + 32 * K + 16) + (D + 1) * (4 + 24)  # + the row
    out = {"bound": "latency (one dependent HBM round trip per tree level, 4 games per wave; pmc.sq: the VALU "
                    "work per launch against its time)",
           "peak_GBps": HBM_PEAK_GBPS, "sims_per_launch": per_launch,
           "kernel": "k_backup_select_seg (expand/backup of simulation s + select of s + 1, one launch per "
                     "simulation step and game part; the first select and the last expand/backup of a move run "
                     "alone)",
           "note": "launch times overlap the other game part's kernels (its NN holds whole CUs), so the rates "
                   "are lower bounds"}
    for name, ms, n, b in (("backup_select", kt.backup_select_ms, kt.backup_select_n, sel + exp),):
        t = ms / n * 1e-3
        gbps = per_launch * b / t / 1e9
        out[name] = {"avg_launch_us": t * 1e6, "algorithmic_bytes_per_sim": b, "achieved_GBps": gbps,
                     "frac": gbps / HBM_PEAK_GBPS}
        if pmc and name in pmc:
            out[name]["pmc"] = dict(pmc[name], note="rocprofv3 FETCH/WRITE_SIZE per simulation over the launches "
                                    "of one steady-state ply (after the warm-up plies); writes are small scattered "
                                    "records (leaf record, counters, path entries), each a whole write transaction. "
                                    "Calibrated (tools/pmc_cal, DESIGN.md section 6): FETCH_SIZE counts 64 B per read "
                                    "request, a request being up to 64 B for a scattered record or a 64-B segment and "
                                    "128 B only for contiguous full-line runs, so fetch_bytes_per_sim (x2) is exact for "
                                    "the runs (a node's children, noise pairs, policy rows) and twice the bytes for the "
                                    "scattered records, fetch_bytes_per_sim_raw the reverse: the kernel's reads lie "
                                    "between the two")
            pm = out[name]["pmc"]
            if "fetch_bytes_per_sim_raw" in pm and "write_bytes_per_sim" in pm:
                lo = (pm["fetch_bytes_per_sim_raw"] + pm["write_bytes_per_sim"]) / b
                hi = (pm["fetch_bytes_per_sim"] + pm["write_bytes_per_sim"]) / b
                pm["traffic_vs_formula"] = [lo, hi]
            sq = out[name]["pmc"].get("sq")
            if sq:  # the launch time the VALU work alone would take, every SIMD issuing VALU every cycle
                sq = dict(sq)
                sq["valu_floor_us_at_nominal_clock"] = sq["valu_cycles_per_simd_per_launch"] / NOMINAL_MHZ
                sq["valu_floor_frac_of_launch"] = sq["valu_floor_us_at_nominal_clock"] / (t * 1e6)
                sq["note"] = ("SQ_INSTS_VALU / SQ_WAVES over the same ply; at 2 issue cycles per wave64 VALU "
                              "instruction (SIMD-32; f64 ops take more) valu_cycles_per_simd_per_launch / clock is a "
                              "lower bound of the launch's VALU time; far below the launch time = latency-bound (the "
                              "launch time here overlaps the other part's kernels, single_stream_launch_us does not)")
                out[name]["pmc"]["sq"] = sq
    return out


def host_cpu():
    """Physical cores this process may use (its CPU affinity, one per (package, core) pair,
    capped by a cgroup CPU quota) and the CPU model: the reference runs one self-play worker per
    core (train.rs:122,147 thread_amnt = available_parallelism; BASELINE.md 4: physical cores)."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        cpus = list(range(os.cpu_count() or 1))
    cores = set()
    for c in cpus:
        try:
            t = Path(f"/sys/devices/system/cpu/cpu{c}/topology")
            cores.add(((t / "physical_package_id").read_text().strip(), (t / "core_id").read_text().strip()))
        except OSError:
            cores.add(("?", str(c)))
    n, how = len(cores), f"{len(cores)} physical cores in the affinity mask ({len(cpus)} logical CPUs)"
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if q != "max" and int(q) // int(per) < n:
            n = max(1, int(q) // int(per))
            how += f", capped by the cgroup CPU quota ({q}/{per})"
    except (OSError, ValueError):
        pass
    share = os.environ.get("OMP_NUM_THREADS")  # the GPU box's CPU share per GPU (16): a pool rule
    if share and share.isdigit() and 0 < int(share) < n:
        n = int(share)
        how += f", capped by this host's CPU share per GPU (OMP_NUM_THREADS={share})"
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, how, model


def cpu_baseline(cfg, seconds, threads):
    """Reference-equivalent CPU baseline: oracle/build/oaz_cpu_baseline plays the
    reference's self-play execution shape — one game per worker thread, workers = physical cores,
    sequential MCTS (the C restatement of mcts_arena.rs), one batch-1 libtorch-CPU (ATen) forward per
    simulation (mcts_arena.rs:267-269 -> net.rs:215-232, the ops tch calls), intra-op threads 1 —
    on a bounded sample of the configuration, plus BASELINE's C1 row (1 game, 50 sims, 1 thread)."""
    from onitama_az.weights import random_weights
    exe = ROOT / "oracle" / "build" / "oaz_cpu_baseline"
    n, how, model = host_cpu()
    threads = threads or n
    with tempfile.TemporaryDirectory() as d:
        wf = Path(d) / f"w{cfg['blocks']}.f32"
        random_weights(0, cfg["blocks"]).astype("float32").tofile(wf)
        run = lambda *a: json.loads(subprocess.run([str(exe), *map(str, a)], capture_output=True, text=True,
                                                   check=True, timeout=600).stdout)
        b = run("bench", wf, cfg["blocks"], cfg["sims"], threads, seconds, cfg["fixed_deck"])
        w3 = Path(d) / "w3.f32"
        random_weights(0, 3).astype("float32").tofile(w3)
        c1 = run("c1", w3, 3, 50)
    return {"value": b["sims_per_s"], "unit": "sims/s", "cores": threads, "kind": "port",
            "games_per_s": b["games_per_s"], "cpu_model": model, "cores_detected": how,
            "sample": f"{b['seconds']:.1f}s of self-play on {threads} worker threads (one game each, searches "
                      f"sequential, batch-1 libtorch-CPU forward per simulation, intra-op threads 1; "
                      f"{cfg['blocks']}-block random-init, {cfg['sims']} sims/move, c_puct 5, root noise): "
                      f"{b['sims']} sims, {b['plies']} plies, {b['games']} games finished",
            "c1": dict(c1, config="BASELINE C1: 1 game, 50 sims/move, 3-block random-init, fixed deck, 1 thread"),
            "implementation": "oracle/cpu_baseline.cpp (C restatement of mcts_arena.rs + ATen CPU ops; the Rust/tch "
                              "binary cannot be built here)"}


TRAIN_METRIC = "training samples/sec (SGD steps of batch 512, forward(train) + alphaloss + backward + SGD)"


def train_flop_per_sample(blocks):
    """forward + input-gradient + weight-gradient dense FLOPs (3x forward, minus the first
    layer's unneeded input gradient)."""
    fwd = FLOP_PER_SIM[blocks] if blocks in FLOP_PER_SIM else 11_681_928 + (blocks - 3) * 3_686_400
    return 3 * fwd - 2 * 25 * 9 * 21 * 64


def train_algorithmic_bytes(blocks, B):
    """HBM-level bytes of one SGD step as the kernels move them (training): every
    activation-sized tensor (R = 25 B rows x 64 fp32 = S bytes) a kernel reads or writes, the weight-gradient
    partials (9 x 25 x 2 tiles of 64 x 64 fp32, written and re-read per layer) and the SGD's parameter,
    gradient and momentum passes. Forward: conv l reads its input (layer 0: 32 of 64 channels) and writes Z,
    the BN apply reads Z (+ the skip at block outputs) and writes A; heads read A (conv) and A, Z (backward
    rows) and write M. Backward per layer: the BN-backward apply reads M, Z and writes dZ; the weight gradient
    reads dZ and the layer input; the input gradient (not for layer 0) reads dZ, the activation, the pre-BN
    output (+ the skip at a block's first conv) and writes M."""
    L = 1 + 2 * blocks
    S = 25 * B * 64 * 4
    fwd = (0.5 + 1.0) * S + (L - 1) * 2.0 * S + L * 2.0 * S + blocks * S
    heads = 4.0 * S
    part = 9 * 25 * 2 * 64 * 64 * 4
    bwd = L * 3.0 * S + (L - 1) * 2.0 * S + 1.5 * S + (L - 1) * 4.0 * S + blocks * S
    bwd += (L - 0.5) * 2.0 * part
    nparam = L * (64 * 64 * 9 + 5 * 64) - 64 * 43 * 9 + 64 + 5 + 64 * 25 + 64 + 64 + 1 + 128 + 10 + 2500 + 50
    return fwd + heads + bwd + 5.0 * 4 * nparam


def pmc_train_traffic(args):
    """FETCH_SIZE / WRITE_SIZE over every trainer kernel of the timed steps, one counter per rocprofv3 pass
    (a child bench process; this process has not touched the GPU yet), summed per SGD step (steps end at
    k_sgd). rocprofv3 serialises the counted dispatches, so the two streams' overlap is gone in these
    passes; bytes per kernel are unaffected. FETCH_SIZE x2 (gfx950 wide-read correction)."""
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    warm, steps = 3, 4
    kb = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        with tempfile.TemporaryDirectory() as d:
            cmd = [prof, "--pmc", ctr, "--kernel-include-regex", "tr::k_", "--output-format", "csv", "-d", d,
                   "-o", "pmc", "--", sys.executable, str(Path(__file__).resolve()), "--mode", "train", "--pmc-child",
                   "--no-cpu-baseline", "--steps", str(steps), "--warmup", str(warm),
                   "--train-blocks", str(args.train_blocks), "--train-batch", str(args.train_batch)]
            try:
                subprocess.run(cmd, timeout=600, capture_output=True, check=True)
            except (subprocess.SubprocessError, OSError) as exc:
                print(f"bench: train PMC pass {ctr} failed ({type(exc).__name__})", file=sys.stderr)
                return None
            rows = []
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if r["Counter_Name"] == ctr:
                        rows.append((int(r.get("Dispatch_Id", 0) or 0), r["Kernel_Name"], float(r["Counter_Value"])))
            rows.sort()
            ends = [i for i, (_, n, _) in enumerate(rows) if "k_sgd" in n]
            if len(ends) < warm + steps:
                print(f"bench: train PMC pass {ctr}: {len(ends)} steps collected", file=sys.stderr)
                return None
            timed = rows[ends[warm - 1] + 1:ends[warm + steps - 1] + 1]
            kb[ctr] = sum(v for _, _, v in timed) / steps
    fetch, write = 2.0 * kb["FETCH_SIZE"] * 1024.0, kb["WRITE_SIZE"] * 1024.0
    return {"bytes_per_step": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
            "fetch_bytes_uncorrected": kb["FETCH_SIZE"] * 1024.0, "raw_kb": kb,
            "note": f"rocprofv3 --pmc, separate passes, every tr::k_ dispatch of {steps} SGD steps after {warm} "
                    "(kernels serialised by the counter collection); FETCH_SIZE x2, the gfx950 correction calibrated "
                    "for 16-byte-per-lane reads (the convs' operand loads); the BN, reduction and SGD kernels read 4 "
                    "bytes per lane, for which it is uncalibrated, so fetch_bytes is an upper bound and "
                    "fetch_bytes_uncorrected a lower one. WRITE_SIZE equals the formula's writes (every intermediate "
                    "tensor once, the weight-gradient partials, the SGD passes)"}


def train_cpu_baseline(blocks, batch, seconds, threads):
    """The reference trains on the CPU through tch (train.rs:163 `Device::Cpu`): the same op graph
    (oracle/train_ref.py) in fp32 ATen on `threads` host threads, batch 512."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import numpy as np
    from train_ref import alphaloss, forward
    from onitama_az.weights import named_from_blob, random_weights
    torch.set_num_threads(threads)
    named = {k: torch.tensor(v, requires_grad=not k.endswith(("running_mean", "running_var")))
             for k, v in named_from_blob(random_weights(0, blocks), blocks).items()}
    params = [t for k, t in named.items() if t.requires_grad]
    opt = torch.optim.SGD(params, lr=5e-3, momentum=0.9, weight_decay=1e-4)
    rng = np.random.default_rng(0)
    x = torch.tensor((rng.random((batch, 21, 5, 5)) < 0.3).astype(np.float32))
    pi = torch.softmax(torch.tensor(rng.normal(size=(batch, 2, 25)).astype(np.float32)).reshape(batch, 50), -1)
    z = torch.tensor(rng.integers(-1, 2, batch).astype(np.float32))
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds or steps < 2:
        opt.zero_grad()
        p, v = forward(named, x, blocks, train=True)
        lv, lp = alphaloss(v, p, pi.reshape(batch, 2, 25), z)
        (lv + lp).backward()
        opt.step()
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": steps * batch / dt, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{steps} SGD steps of batch {batch} in {dt:.1f}s: fp32 ATen on {threads} host threads "
                      f"(oracle/train_ref.py op graph = net.rs forward(train) + alphaloss + tch SGD), {blocks}-block"}


def train_main(args, world, rank, local):
    import numpy as np
    from onitama_az import _abi
    from onitama_az.game import initial_state_np
    from onitama_az.trainer import Trainer, _DeviceArray, choose_batches
    from onitama_az.weights import random_weights
    blocks, B = args.train_blocks, args.train_batch
    assert B % world == 0 and (B // world) % 16 == 0, "per-rank batch must be a multiple of 16"
    traffic = None
    if not args.pmc_child and not args.no_pmc and world == 1:
        traffic = pmc_train_traffic(args)  # child processes, before this process touches the GPU
    shard = B // world
    lib = _abi.load()
    n_samples = 65536
    rng = np.random.default_rng(rank)
    deals = np.zeros((n_samples, 5), dtype=np.uint8)
    for g in range(n_samples):  # seeded 5-of-16 deals, as the self-play engine deals them
        import ctypes as C
        d = (C.c_uint8 * 5)()
        lib.oaz_deal_deck(C.c_uint64(20260101), C.c_uint64(g), d)
        deals[g] = list(d)
    samples = np.zeros(n_samples, dtype=_abi.SAMPLE_DTYPE)
    samples["state"] = np.concatenate([initial_state_np(deals[g]) for g in range(n_samples)])
    pi = rng.random((n_samples, 50)).astype(np.float32)
    samples["pi"] = pi / pi.sum(1, keepdims=True)
    samples["z"] = rng.integers(-1, 2, n_samples).astype(np.float32)
    tr = Trainer(blocks=blocks, max_batch=shard, device=local)
    tr.set_weights(random_weights(0, blocks))
    ts = torch.cuda.Stream()  # explicit: handle 0 would leave the trainer on its own, unordered stream
    torch.cuda.set_stream(ts)
    tr.set_stream(ts.cuda_stream)
    tr.load_samples(samples)
    nb = args.warmup + args.steps
    idx = choose_batches(np.random.default_rng(1), n_samples, B, nb)[:, rank * shard:(rank + 1) * shard]
    tr.set_batches(idx)
    grads = None
    if world > 1:
        ptr, n = tr.grads_device()
        grads = torch.as_tensor(_DeviceArray(ptr, n), device=f"cuda:{local}")

    def step(b):
        if world > 1:
            tr.backward(b)
            dist.all_reduce(grads)
            tr.apply(1.0 / world)
        else:
            tr.train(b, 1)

    def barrier_sync():
        torch.cuda.synchronize()
        tr.sync()
        if world > 1:
            dist.barrier()

    for b in range(args.warmup):
        step(b)
    barrier_sync()
    t0 = time.perf_counter()
    for b in range(args.warmup, nb):
        step(b)
    t_enq = time.perf_counter() - t0  # the host's enqueue time of the K steps (the device may still be running)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    tmax = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    T = float(tmax.item())
    v, p, k = tr.losses()
    if rank == 0:
        fl = train_flop_per_sample(blocks) * shard
        ms = 1e3 * T / args.steps
        achieved = fl / (ms * 1e-3) / 1e12
        out = {"metric": TRAIN_METRIC, "value": B * args.steps / T, "unit": "samples/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
               "data": "synthetic (seeded deals, random pi/z, random-init weights seed 0)",
               "config": {"workload": f"train: {blocks}-block ResNet, global batch {B}, lr 5e-3, momentum 0.9, "
                                      f"wd 1e-4", "parallelism": f"dp{world} (RCCL all-reduce of gradients)"},
               "mean_losses": {"value": v / max(1, k), "policy": p / max(1, k)},
               "host_enqueue_ms_per_step": 1e3 * t_enq / args.steps,
               "roofline": {"bound": "mfma", "kernel": "whole SGD step (conv fwd/dgrad/wgrad on v_mfma_f32_16x16x4_f32)",
                            "achieved": achieved, "peak": PEAK_TFLOPS["fp32"], "unit": "TFLOP/s",
                            "frac": achieved / PEAK_TFLOPS["fp32"],
                            "traffic": traffic["bytes_per_step"] if traffic else None,
                            "traffic_unit": "HBM-side bytes per SGD step (PMC)",
                            "algorithmic_bytes_per_step": train_algorithmic_bytes(blocks, shard),
                            "traffic_detail": traffic,
                            "flop_per_step_per_gpu": fl}}
        if not args.no_cpu_baseline and world == 1:
            try:  # after the timed region: a baseline failure must not lose the measured line
                out["cpu_baseline"] = train_cpu_baseline(blocks, B, args.cpu_seconds,
                                                         args.cpu_threads or min(16, os.cpu_count() or 1))
            except Exception as ex:  # noqa: BLE001
                print(f"bench: cpu_baseline failed: {ex!r}", file=sys.stderr, flush=True)
                out["cpu_baseline"] = {"error": repr(ex)}
        print(json.dumps(out), flush=True)
    tr.close()
    if world > 1:
        dist.destroy_process_group()


PM_METRIC = "pure-MCTS playouts/sec (random-rollout UCT agent, onitama-game ai/mcts)"


def pmc_pure_mcts(args):
    """k_pure_mcts's VALU issue against the SIMDs' issue peak: one child pass `rocprofv3 --pmc SQ_INSTS_VALU
    SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace` over one search of the bench's workload (one launch; this process
    has not touched the GPU yet). achieved = wave64 VALU instructions / the traced duration; peak = 1 024 SIMDs x
    2.4 GHz / 2 cycles per wave64 instruction (SIMD-32); GRBM_GUI_ACTIVE / 8 XCDs / duration = the clock."""
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    with tempfile.TemporaryDirectory() as d:
        cmd = [prof, "--pmc", "SQ_INSTS_VALU", "SQ_WAVES", "GRBM_GUI_ACTIVE", "--kernel-trace",
               "--kernel-include-regex", "k_pure_mcts", "--output-format", "csv", "-d", d, "-o", "pm", "--",
               sys.executable, str(Path(__file__).resolve()), "--mode", "pure_mcts", "--pmc-child", "--no-cpu-baseline",
               "--steps", "1", "--warmup", "1", "--pm-games", str(args.pm_games), "--pm-playouts", str(args.pm_playouts)]
        try:
            subprocess.run(cmd, timeout=600, capture_output=True, check=True)
        except (subprocess.SubprocessError, OSError) as exc:
            print(f"bench: pure-MCTS PMC pass failed ({type(exc).__name__})", file=sys.stderr)
            return None
        ctr, dur = {}, {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_pure_mcts" in r["Kernel_Name"]:
                    k = (int(r["Dispatch_Id"]), r["Counter_Name"])
                    ctr[k] = ctr.get(k, 0.0) + float(r["Counter_Value"])
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_pure_mcts" in r["Kernel_Name"]:
                    dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    ids = sorted(set(i for i, _ in ctr) & set(dur))
    if not ids:
        print("bench: pure-MCTS PMC pass collected no k_pure_mcts rows", file=sys.stderr)
        return None
    i = ids[-1]  # the timed search (after the warm-up one)
    valu, waves, t = ctr.get((i, "SQ_INSTS_VALU"), 0.0), ctr.get((i, "SQ_WAVES"), 0.0), dur[i]
    clock = ctr.get((i, "GRBM_GUI_ACTIVE"), 0.0) / XCDS / t / 1e6 if t > 0 else 0.0
    peak = SIMDS * NOMINAL_MHZ * 1e6 / VALU_CYC
    achieved = valu / t if t > 0 else 0.0
    return {"bound": "valu", "kernel": "k_pure_mcts (one thread per search, rollouts: attack-table lookups, popcounts, "
                                       "Philox draws)",
            "achieved": achieved / 1e9, "peak": peak / 1e9, "unit": "G wave64 VALU instructions/s",
            "frac": achieved / peak, "traffic": None,
            "frac_at_measured_clock": achieved / (SIMDS * clock * 1e6 / VALU_CYC) if clock > 0 else None,
            "measured_clock_mhz": clock, "valu_instructions_per_wave": valu / waves if waves else None,
            "profiled_launch_ms": t * 1e3,
            "note": "rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace, one search launch after a "
                    "warm-up one; instructions are counted per wave, so lanes idled by divergent rollout lengths "
                    "still count as issued: frac is an upper bound of the lane-level utilisation; traffic is null "
                    "(the trees and the attack table stay in L2 / LDS; the bound is issue, not memory)"}


def pure_mcts_main(args, world, rank, local):
    """One step = one search (max_playouts random-rollout playouts) from each of pm_games seeded
    deals (the arena opponent's config: min_node_visits 5, c 1.41, evaluator.rs:340-345)."""
    import ctypes as C
    import numpy as np
    from onitama_az import _abi
    from onitama_az.game import initial_state_np
    from onitama_az.pure_mcts import pure_mcts_search
    G, P = args.pm_games, args.pm_playouts
    roof = None
    if not args.pmc_child and not args.no_pmc and world == 1:
        roof = pmc_pure_mcts(args)  # a child process, before this process touches the GPU
    lib = _abi.load()
    deals = []
    for g in range(G):
        d = (C.c_uint8 * 5)()
        lib.oaz_deal_deck(C.c_uint64(20260101), C.c_uint64(rank * G + g), d)
        deals.append(initial_state_np(list(d)))
    roots = np.concatenate(deals)

    def step(k):
        return pure_mcts_search(roots, P, 5, 1.41, seed=20260101, game_id0=(k * world + rank) * G)

    for k in range(args.warmup):
        step(k)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    plies = 0
    for k in range(args.steps):
        r = step(args.warmup + k)
        plies += r.stats.rollout_plies
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tmax = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    T = float(tmax.item())
    if rank == 0:
        total = G * P * args.steps * world
        out = {"metric": PM_METRIC, "value": total / T, "unit": "playouts/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": 1e3 * T / args.steps, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "int32/f32",
               "data": "synthetic (seeded 5-of-16 deals, start positions)",
               "config": {"workload": f"pure_mcts: {G} searches/GPU x {P} playouts, min_node_visits 5, c 1.41",
                          "parallelism": f"searches sharded x{world}"},
               "searches_per_s": G * args.steps * world / T,
               "mean_rollout_plies": plies / max(1, G * P * args.steps), "roofline": roof}
        if not args.no_cpu_baseline and world == 1:
            try:  # after the timed region: a baseline failure must not lose the measured line
                sys.path.insert(0, str(ROOT / "tests"))
                import oracle_ffi as orc
                from onitama_az.pure_mcts import default_config
                cfg = default_config()
                cfg.max_playouts, cfg.min_node_visits, cfg.exploration_c = P, 5, 1.41
                threads = args.cpu_threads or min(16, os.cpu_count() or 1)
                t1 = time.perf_counter()
                po, ns = orc.pure_mcts_bench(cfg, threads, args.cpu_seconds)
                dt = time.perf_counter() - t1
                out["cpu_baseline"] = {"value": po / dt, "unit": "playouts/s", "cores": threads, "kind": "port",
                                       "sample": f"{ns} searches x {P} playouts in {dt:.1f}s on {threads} host "
                                                 f"threads (oracle C restatement of mcts_arena.rs)"}
            except Exception as ex:  # noqa: BLE001
                print(f"bench: cpu_baseline failed: {ex!r}", file=sys.stderr, flush=True)
                out["cpu_baseline"] = {"error": repr(ex)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


ARENA_METRIC = "arena fight games/sec (AlphaZero vs AlphaZero, evaluator.rs fight, 400 sims/move, train=false)"


def arena_main(args, world, rank, local):
    """one step = one whole fight (evaluator.rs:355-399) of arena_games games between
    two AlphaZero agents (3-block random-init weights, seeds 0 and 1; AlphaZeroMctsConfig of the pit,
    evaluator.rs:198-204, with the playout budget and no time cutoff), the games played in parallel
    (onitama_az/evaluator.py fight: every ply, each agent searches all of its games in one batched
    oaz_search). Games are sharded over ranks (each rank its own deals); nothing is exchanged."""
    from onitama_az import _abi
    from onitama_az.evaluator import AlphaZeroAgent, EvaluatorConfig, fight
    from onitama_az.mcts import AlphaZeroMctsConfig, ConvResNet, ConvResNetConfig, Options
    n, sims = args.arena_games, args.sims or 400
    opts = Options(precision=_abi.FP32_SPLIT16, device=local)
    net = ConvResNetConfig(resnet_block_amnt=3)
    new, best = ConvResNet(net, opts, seed=0), ConvResNet(net, opts, seed=1)
    # exactly `sims` playouts per move (a 131 072-game batch would pass the reference's 400 ms per-agent budget,
    # which is a per-game clock in the reference, as one batch clock)
    cfg = AlphaZeroMctsConfig(search_time=0.4, exploration_c=5.0, max_playouts=sims, train=False,
                              enforce_search_time=False)
    agent, opponent = AlphaZeroAgent(cfg, new), AlphaZeroAgent(cfg, best)
    fight(EvaluatorConfig(game_amnt=n, max_plies=1, seed=20260101 + rank), agent, opponent)  # warm-up: 3 plies
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    plies = games = 0
    wins = [0, 0, 0]
    for k in range(args.steps):
        st = fight(EvaluatorConfig(game_amnt=n, seed=20260101 + (k + 1) * world + rank), agent, opponent)
        plies += sum(st.plies)
        games += n
        wins[0] += st.general.wins
        wins[1] += st.general.loses
        wins[2] += st.general.draws
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    cdev = "cpu" if os.environ.get("OAZ_BENCH_REHEARSE") == "1" else "cuda"  # (gloo rehearsal: host tensors)
    t = torch.tensor([elapsed, float(plies), float(games)], dtype=torch.float64, device=cdev)
    if world > 1:
        tm = t[:1].clone()
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t[0] = tm[0]
    T, plies_all, games_all = (float(x) for x in t.tolist())
    if rank == 0:
        out = {"metric": ARENA_METRIC, "value": games_all / T, "unit": "games/s", "n_gpus": world, "steps": args.steps,
               "warmup": 1, "ms_per_step": 1e3 * T / args.steps, "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "fp32 (fp16x3 split)",
               "data": "synthetic (random-init weights seeds 0 / 1, seeded 5-of-16 deals)",
               "config": {"workload": f"arena: {n} games/GPU per fight, {sims} sims/move, 3-block, c 5, train=false, "
                                      "152-ply cut", "parallelism": f"games sharded x{world}"},
               "sims_per_s": plies_all * sims / T, "plies_per_s": plies_all / T,
               "mean_plies_per_game": plies_all / max(1.0, games_all),
               "rank0_results": {"wins": wins[0], "loses": wins[1], "draws": wins[2]},
               "note": "a fight runs until its last game ends (or the 152-ply cut), so its tail searches few games"}
        if not args.no_cpu_baseline and world == 1:
            try:
                cb = cpu_baseline({"blocks": 3, "sims": sims, "fixed_deck": 0}, args.cpu_seconds, args.cpu_threads)
                mpg = out["mean_plies_per_game"]
                out["cpu_baseline"] = {"value": cb["value"] / (sims * mpg), "unit": "games/s", "cores": cb["cores"],
                                       "kind": "port", "sims_per_s": cb["value"],
                                       "sample": cb["sample"] + f"; games/s = sims/s / ({sims} sims x {mpg:.1f} plies "
                                                 "per game of this fight); the reference's arena runs the same "
                                                 "searches without root noise (train=false)"}
            except Exception as ex:  # noqa: BLE001
                out["cpu_baseline"] = {"error": repr(ex)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def sim_parts(games, parts=0):
    """Game parts (streams) of the engine's simulation loop: oaz_config.parts, or auto = 2 from 2048
    games (oaz_engine.cpp game_parts); bench.py checks it against kernel_times().parts."""
    return parts if parts in (1, 2, 4) else (2 if games >= 2048 else 1)


def nn_step_rate(kt, evals, sim_steps, blocks):
    """The NN's rate per simulation step. Each step launches the NN once per game part (kt.parts,
    one stream each); the parts' launches overlap, so a step's NN time is the union of their
    intervals (kt.nn_busy_ms over the timed steps), and its positions are all game slots
    (kt.nn_samples, counted by the engine) or, with leaf compaction, the leaves the playouts use
    (nn_evals over the region / its simulation steps)."""
    parts = max(1, kt.parts)
    steps_timed = max(1, kt.nn_n // parts)
    positions = kt.nn_samples / steps_timed if kt.nn_samples else evals / max(1, sim_steps)
    busy = kt.nn_busy_ms / steps_timed
    flops = FLOP_PER_SIM[blocks] * positions
    return {"parts": parts, "positions": positions, "busy_ms": busy, "flops": flops,
            "avg_launch_ms": kt.nn_ms / max(1, kt.nn_n),
            "achieved": flops / (busy * 1e-3) / 1e12 if kt.nn_n and busy > 0 else 0.0}


PREC_ABI = {"bf16": "BF16", "fp32": "FP32", "fp32_split": "FP32_SPLIT", "fp32_split16": "FP32_SPLIT16"}


def single_stream_leg(args, cfg, device, precision):
    """The workload on one stream (oaz_config.parts = 1), a short run (2 warm-up + 2 timed plies, no
    staggered starts) with HIP events around the NN launches of every 8th simulation step on the
    engine stream. With the headline's two game parts the parts' NN launches overlap each other
    and the other part's tree kernels, so per-launch event times there include waiting for CUs;
    here every launch has the GPU to itself, which is what a kernel roofline needs."""
    from onitama_az import _abi
    from onitama_az.engine import Engine
    from onitama_az.weights import random_weights
    with Engine(device=device, games=cfg["games"], sims=cfg["sims"], blocks=cfg["blocks"], c_puct=5.0,
                train_noise=0 if args.no_noise else 1, max_plies=150, evaluator=_abi.EVAL_NN,
                precision=getattr(_abi, PREC_ABI[precision]), fixed_deck=cfg["fixed_deck"], deck=[0, 1, 2, 3, 4],
                seed=20260101, sample_capacity=cfg["games"] * 8, parts=1, compact=0, step_kernels=1) as e:
        e.load_weights(random_weights(0, cfg["blocks"]))
        e.selfplay_reset()
        e.selfplay_step(2)
        e.sync()
        st0 = e.selfplay_stats()
        e.kernel_times_reset()
        e.set_timing(8)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.selfplay_step(2)
        e.sync()
        dt = time.perf_counter() - t0
        e.set_timing(False)
        kt = e.kernel_times()
        st1 = e.selfplay_stats()
    sims = st1.search.sims - st0.search.sims
    nn = nn_step_rate(kt, st1.search.nn_evals - st0.search.nn_evals, 2 * cfg["sims"], cfg["blocks"])
    nn["nonzero_achieved"] = (nonzero_flop_per_sim(cfg["blocks"]) * nn["positions"] / (nn["avg_launch_ms"] * 1e-3)
                              / 1e12 if nn["avg_launch_ms"] > 0 else 0.0)
    nn.update(sims_per_s=sims / dt, ms_per_step=1e3 * dt / 2, launches=kt.nn_n,
              tree_launch_us=1e3 * kt.backup_select_ms / kt.backup_select_n if kt.backup_select_n else None)
    return nn


def compaction_leg(args, cfg, device, stagger):
    """The headline workload with leaf compaction on (oaz_config.compact = 2): the leaves whose
    evaluation the reference computes and discards (a won, terminal-flagged leaf: no expansion, the
    reward is backed up, mcts_arena.rs:156-176) do not go to the network. The trees, pi and samples
    are those of the headline run; the headline itself keeps one NN evaluation per playout (the
    metric's unit of work). Same warm-up and staggered starts, 2 timed plies."""
    from onitama_az import _abi
    from onitama_az.engine import Engine
    from onitama_az.weights import random_weights
    with Engine(device=device, games=cfg["games"], sims=cfg["sims"], blocks=cfg["blocks"], c_puct=5.0,
                train_noise=0 if args.no_noise else 1, max_plies=150, evaluator=_abi.EVAL_NN,
                precision=getattr(_abi, PREC_ABI[cfg["precision"]]), fixed_deck=cfg["fixed_deck"],
                deck=[0, 1, 2, 3, 4], seed=20260101, sample_capacity=cfg["games"] * (args.warmup + 4),
                stagger=stagger, compact=2) as e:
        e.load_weights(random_weights(0, cfg["blocks"]))
        e.selfplay_reset()
        e.selfplay_step(args.warmup)
        e.sync()
        st0 = e.selfplay_stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.selfplay_step(2)
        e.sync()
        dt = time.perf_counter() - t0
        st1 = e.selfplay_stats()
        kt = e.kernel_times()
    sims = st1.search.sims - st0.search.sims
    evals = st1.search.nn_evals - st0.search.nn_evals
    return {"value": sims / dt, "unit": "sims/s", "ms_per_step": 1e3 * dt / 2, "steps": 2, "warmup": args.warmup,
            "nn_positions_per_sim": evals / max(1, sims), "game_parts": kt.parts,
            "note": "oaz_config.compact = 2: a won, terminal-flagged leaf's evaluation (computed and discarded by "
                    "the reference) is not sent to the network; identical trees / pi / samples (GPU parity tests "
                    "run both settings); not the headline, whose unit of work includes every leaf evaluation"}


def exact_fp32_leg(args, cfg, device):
    """The same workload on the exact-fp32 NN kernel (k_nn_sq16: fp32 MFMA products), so the
    headline's precision trade is visible in the same line (single_stream_leg)."""
    nn = single_stream_leg(args, cfg, device, "fp32")
    return {"kernel": NN_KERNEL["fp32"], "value": nn["sims_per_s"], "unit": "sims/s", "ms_per_step": nn["ms_per_step"],
            "steps": 2, "warmup": 2, "game_parts": 1, "nn_avg_launch_ms": nn["avg_launch_ms"],
            "nn_achieved_TFLOPs": nn["achieved"], "nn_frac_of_fp32_mfma_peak": nn["achieved"] / PEAK_TFLOPS["fp32"],
            "note": "same workload on one stream, exact fp32 MFMA products (no operand splitting); short run "
                    "without staggered starts (the NN dominates the step)"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # OAZ_BENCH_REHEARSE=1: every rank on GPU 0 with gloo collectives (exercises the multi-rank path
    # of this script on a one-GPU box; its timings mean nothing)
    rehearse = os.environ.get("OAZ_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if args.mode == "train":
        return train_main(args, world, rank, local)
    if args.mode == "pure_mcts":
        return pure_mcts_main(args, world, rank, local)
    if args.mode == "arena":
        return arena_main(args, world, rank, local)
    from onitama_az import _abi
    from onitama_az.engine import Engine
    from onitama_az.weights import random_weights

    cfg = dict(CONFIGS[args.config])
    if cfg["precision"] == "fp32" and args.fp32_kernel in ("split", "split16"):
        cfg["precision"] = {"split": "fp32_split", "split16": "fp32_split16"}[args.fp32_kernel]
    if args.games:
        cfg["games"] = args.games
    if args.sims:
        cfg["sims"] = args.sims
    # staggered starts must be over before the timed region (every slot playing)
    stagger = min(args.stagger, args.warmup) if args.stagger > 1 else 0
    traffic = clock = None
    if not args.pmc_child and not args.no_pmc and world == 1:
        traffic = pmc_traffic(args, cfg)  # child processes; this process has not touched the GPU yet
        clock = pmc_clock(args, cfg)
    eng = Engine(device=local, games=cfg["games"], sims=cfg["sims"], blocks=cfg["blocks"], c_puct=5.0,
                 train_noise=0 if args.no_noise else 1,
                 max_plies=150, evaluator=_abi.EVAL_NN,
                 precision={"bf16": _abi.BF16, "fp32_split": _abi.FP32_SPLIT,
                            "fp32_split16": _abi.FP32_SPLIT16}.get(cfg["precision"], _abi.FP32),
                 fixed_deck=cfg["fixed_deck"],
                 deck=[0, 1, 2, 3, 4], seed=20260101, rank=rank, world=world,
                 # every sample of every game that can finish in warmup + steps plies fits (checked below)
                 sample_capacity=cfg["games"] * (max(args.warmup, args.pmc_plies) + args.steps + 2), stagger=stagger,
                 compact=0,  # every playout evaluates its leaf: the metric's unit of work
                 parts=args.pmc_parts if args.pmc_child else 0)
    eng.load_weights(random_weights(0, cfg["blocks"]))  # random-init weights (seed 0), SURVEY.md 8d
    eng.selfplay_reset()
    if args.pmc_child:  # profiled pass: the warm-up plies (not collected), then one collected ply
        for _ in range(args.pmc_plies + 1):
            eng.selfplay_step(1)
        eng.sync()
        eng.close()
        return

    def barrier_sync():
        torch.cuda.synchronize()
        eng.sync()
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        eng.selfplay_step(1)
    barrier_sync()
    st0 = eng.selfplay_stats()
    eng.kernel_times_reset()
    # HIP events around the kernels of every 8th simulation step: an event pair around every launch
    # costs ~2 % of the step (measured), sampling keeps the live per-kernel averages nearly free
    eng.set_timing(int(os.environ.get("OAZ_BENCH_TIMING_EVERY", "8")))
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.selfplay_step(1)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    eng.set_timing(False)
    kt = eng.kernel_times()
    st1 = eng.selfplay_stats()

    sims = st1.search.sims - st0.search.sims
    evals = st1.search.nn_evals - st0.search.nn_evals  # leaves sent to the network (compacted)
    games_done = st1.games_finished - st0.games_finished
    plies = st1.moves - st0.moves
    expansions = st1.search.expansions - st0.search.expansions
    depth = (st1.search.depth_sum - st0.search.depth_sum) / max(1, sims)
    branching = (st1.search.children - st0.search.children) / max(1, expansions)
    cdev = "cpu" if rehearse else "cuda"
    fallbacks = eng.nn_fallbacks()
    tot = torch.tensor([float(sims), float(games_done), float(plies), float(expansions), float(st1.samples_dropped),
                        float(fallbacks)], dtype=torch.float64, device=cdev)
    tmax = torch.tensor([elapsed, float(st1.search.max_nodes)], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    sims_all, games_all, plies_all, exp_all, dropped_all, fallbacks_all = (float(x) for x in tot.tolist())
    T, max_nodes_all = (float(x) for x in tmax.tolist())

    # validity of the measured run over all ranks (the process exits non-zero if a check fails):
    # no sample lost to the device buffer, no tree beyond its capacity, every rank simulated
    cap_nodes = 1 + 40 * cfg["sims"]
    checks = {"samples_dropped": int(dropped_all), "max_nodes": int(max_nodes_all), "tree_capacity": cap_nodes,
              "nn_fp16_range_fallback_tiles": int(fallbacks_all),
              "ok": bool(dropped_all == 0 and max_nodes_all <= cap_nodes and sims_all > 0)}

    # per-rank view of the timed region for the line: every rank's simulations and time (rank order)
    per_rank = torch.tensor([float(st1.search.sims - st0.search.sims), elapsed], dtype=torch.float64, device=cdev)
    if world > 1:
        gathered = [torch.zeros_like(per_rank) for _ in range(world)]
        dist.all_gather(gathered, per_rank)
    else:
        gathered = [per_rank]
    rank_sims = [float(t[0]) for t in gathered]
    rank_s = [float(t[1]) for t in gathered]

    allgather = None
    if not args.no_allgather:  # C4: RCCL all-gather of (s, pi, z) after the timed region
        from onitama_az.dist import Comm, allgather_sample_bytes, allgather_samples_device
        comm = None
        # after the timed region: an exchange error is reported in the line (and on stderr) instead
        # of losing the measured throughput with it
        try:
            if rehearse:  # gloo over host copies (one-GPU rehearsal of the multi-rank script)
                t1 = time.perf_counter()
                mine = eng.samples_fetch(int(eng.selfplay_stats().samples_ready))
                own = len(mine)
                raw = allgather_sample_bytes(torch.from_numpy(mine.view("uint8").copy()), world)
                total, counts = raw.numel() // 228, None
                allgather = {"backend": "gloo (rehearsal, host copies)", "seconds": time.perf_counter() - t1}
            else:
                with _StdoutToStderr():
                    comm = Comm.create(rank, world, local)
                    raw, total, counts = allgather_samples_device(eng, world, torch.device("cuda", local), comm)
                    torch.cuda.synchronize()
                cs = comm.stats()
                own = int(cs.own_records)
                recv = (total - own) * 228  # bytes this rank received over the links
                allgather = {"backend": "oaz_allgather_samples (C ABI: RCCL counts all-gather + grouped broadcasts)",
                             "rccl_ranks": int(cs.ranks), "counts": counts, "collective_ms": cs.allgather_ms,
                             "counts_ms": cs.counts_ms, "bytes_received": recv,
                             "GBps_received": recv / (cs.allgather_ms * 1e-3) / 1e9 if cs.allgather_ms > 0 else None,
                             "xgmi_note": f"xGMI: {XGMI_LINK_GBPS:.0f} GB/s per link and direction, 7 links per GPU; "
                                          "collective_ms = HIP events on the communicator stream around the grouped "
                                          "broadcasts only (no host copies)"}
        except Exception as ex:  # noqa: BLE001
            print(f"bench: sample all-gather failed on rank {rank}: {ex!r}", file=sys.stderr, flush=True)
            allgather = {"error": repr(ex)}
        if comm is not None:
            comm.close()
        # The post-processing collectives run only when every rank's exchange succeeded: every rank joins
        # this status reduction first (also a rank whose exchange raised), so no rank waits in a later
        # collective that another skipped.
        all_ok = "error" not in allgather
        if world > 1:
            okt = torch.tensor([1.0 if all_ok else 0.0], dtype=torch.float64, device=cdev)
            dist.all_reduce(okt, op=dist.ReduceOp.MIN)
            all_ok = bool(okt.item() == 1.0)
        if all_ok:
            # every rank: the gathered total is the sum of the ranks' own contributions
            chk = torch.tensor([float(own), float(total)], dtype=torch.float64, device=cdev)
            ms = torch.tensor([allgather.get("collective_ms", 0.0)], dtype=torch.float64, device=cdev)
            if world > 1:
                dist.all_reduce(chk[:1])
                dist.all_reduce(ms, op=dist.ReduceOp.MAX)
            ok = int(chk[0].item()) == total and (counts is None or sum(counts) == total)
            if world > 1:
                okt = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=cdev)
                dist.all_reduce(okt, op=dist.ReduceOp.MIN)
                ok = bool(okt.item() == 1.0)
            allgather.update(samples_total=int(total), bytes_per_sample=228, totals_consistent=ok)
            if world > 1 and "collective_ms" in allgather:
                allgather["collective_ms_max_over_ranks"] = float(ms.item())
            if not ok:
                print(f"bench: all-gather totals inconsistent on rank {rank}", file=sys.stderr, flush=True)
        elif "error" not in allgather:
            allgather["error"] = "another rank's exchange failed"

    if rank == 0:
        sims_steps = cfg["sims"]  # simulation steps (select -> NN -> expand launches) per bench step
        nn = nn_step_rate(kt, evals, args.steps * sims_steps, cfg["blocks"])
        parts, positions, achieved = nn["parts"], nn["positions"], nn["achieved"]
        if traffic and "game_parts" in traffic and parts != sim_parts(cfg["games"]):
            print(f"bench: PMC passes assumed {sim_parts(cfg['games'])} game parts, the run used {parts}",
                  file=sys.stderr)
        out = {
            "metric": METRIC, "value": sims_all / T, "unit": "sims/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * T / args.steps, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"bf16": "bf16", "fp32": "fp32", "fp32_split": "fp32 (bf16x6 split)",
                      "fp32_split16": "fp32 (fp16x3 split)"}[cfg["precision"]],
            "nn_arithmetic": {"fp32": "exact fp32 MFMA products, fp32 accumulate",
                              "fp32_split": "fp32 operands split exactly into hi+mid+lo bf16 terms, the 6 products "
                                            "above 2^-24 relative on bf16 MFMA, fp32 accumulate (error vs float64 = "
                                            "the exact-fp32 kernel's; tests/test_gpu.py 1e-4 parity)",
                              "fp32_split16": "fp32 operands split into hi = fp16(x) and lo = fp16(x - hi) (weights "
                                              "pre-scaled per output channel by a power of two), the 3 products "
                                              "hi*hi, hi*lo, lo*hi on fp16 MFMA, fp32 accumulate (within 1e-5 of the "
                                              "fp32 goldens, tests/test_gpu.py); a 16-position tile whose activations "
                                              "leave the fp16 range is recomputed in-kernel with the bf16x6 split "
                                              "(counted in checks.nn_fp16_range_fallback_tiles)",
                              "bf16": "bf16 MFMA inputs, fp32 accumulate"}[cfg["precision"]],
            "data": "synthetic (random-init weights seed 0, seeded deals)",
            "config": {"workload": f"{args.config}: {cfg['games']} self-play games/GPU x {cfg['sims']} sims/move, "
                                   f"{cfg['blocks']}-block 64-ch ResNet, c_puct 5, Dirichlet root noise",
                       "games_per_gpu": cfg["games"], "sims_per_move": cfg["sims"], "blocks": cfg["blocks"],
                       "fixed_deck": bool(cfg["fixed_deck"]), "parallelism": f"games sharded x{world}"},
            "sims_per_s_per_gpu": sims_all / T / world, "stagger": stagger,
            "games_per_s": games_all / T, "plies_per_s": plies_all / T,
            "true_expansions_per_s": exp_all / T, "mean_select_depth": depth, "mean_branching": branching,
            "plies_per_game": plies_all / max(1.0, games_all),  # steady state: plies played per game finished
            "nn_positions_per_sim": positions * args.steps * sims_steps / max(1, sims),
            "game_parts": parts,
            "nn_leaf_evaluations": "every playout" if kt.nn_samples else "compacted",
            "nn_evaluation": "one NN evaluation per simulation, terminal leaves included (Q2, the metric's unit of "
                             "work: SURVEY 8d); the leaf_compaction block measures the same workload with the "
                             "evaluations the reference discards left out (oaz_config.compact)",
            "kernel_ms_per_step": {
                "backup_select_fused": kt.backup_select_ms / max(1, kt.backup_select_n) * (sims_steps - 1),
                "select_first": kt.select_ms / max(1, kt.select_n) if kt.select_n else None,
                "expand_backup_last": kt.expand_ms / max(1, kt.expand_n) if kt.expand_n else None,
                "nn": nn["busy_ms"] * sims_steps,
                "leaf_compact": kt.compact_ms / max(1, kt.compact_n) * sims_steps,
                "move": kt.finalize_ms / args.steps, "root_noise_stream2": kt.noise_ms / args.steps},
            "kernel_timing": "HIP events around the kernels of every %s-th simulation step (per-kernel means x "
                             "simulation steps per bench step; nn: the union of the game parts' overlapping NN "
                             "launches per step; the tree kernels' launches overlap the other part's too)"
                             % os.environ.get("OAZ_BENCH_TIMING_EVERY", "8"),
            "nn_in_loop": {"game_parts": parts, "busy_ms_per_sim_step": nn["busy_ms"],
                           "avg_launch_ms": nn["avg_launch_ms"], "positions_per_sim_step": positions,
                           "achieved_TFLOPs": achieved,
                           "note": "the game parts' NN launches of a simulation step overlap each other and the "
                                   "other part's tree kernels; busy = the union of their HIP-event intervals, "
                                   "which includes waiting for CUs (the roofline below is measured on one stream)"},
            "tree_kernels": tree_roofline(kt, sims, args.steps * sims_steps, expansions, depth, branching, cfg,
                                          traffic.get("tree_pmc") if traffic else None),
            "allgather": allgather,
            "ranks": {"world": world, "sims_per_rank": rank_sims, "seconds_per_rank": rank_s,
                      "min_rank_s": min(rank_s), "max_rank_s": max(rank_s),
                      "note": "value = all ranks' simulations / the max rank time (barrier + synchronize on both sides)"},
            "checks": checks,
        }
    eng.close()
    # Up to 16 x CU-count games (C2) the engine runs each root-noise chunk (up to 512 simulations: a C2 ply)
    # as ONE launch of k_search_grp (16 games per workgroup: tree walks, k_nn_h3's body, backups); its launches are then
    # the timed region's dominant kernel (kernel class backup_select, every launch timed).
    grp_mode = kt.select_n == 0 and kt.nn_n == 0 and kt.backup_select_n > 0
    if rank == 0 and grp_mode:
        own_sims = st1.search.sims - st0.search.sims
        per_launch = own_sims / kt.backup_select_n
        avg_ms = kt.backup_select_ms / kt.backup_select_n
        flops = FLOP_PER_SIM[cfg["blocks"]] * per_launch
        out["search_kernel"] = {
            "kernel": "k_search_grp (16 games per workgroup: select -> k_nn_h3 body -> expand/backup for one "
                      "root-noise chunk of up to 512 simulations per launch; oaz_search_lat.hip)",
            "launches": kt.backup_select_n, "avg_launch_ms": avg_ms, "sims_per_launch": per_launch,
            "achieved_TFLOPs": flops / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0}
        # k_search_grp evaluates every leaf row of its 16-game tile at every simulation (terminal leaves and
        # slots still waiting for a staggered start included): G positions per simulation step, not the
        # GS_EVALS count of the evaluations the playouts use
        out["nn_positions_per_sim"] = cfg["games"] * args.steps * cfg["sims"] / max(1, own_sims)
        out["nn_leaf_evaluations"] = "every playout (k_search_grp: every leaf row of its 16-game tile)"
        for k in ("backup_select_fused", "nn"):
            out["kernel_ms_per_step"].pop(k, None)
        out["kernel_ms_per_step"]["search_grp"] = kt.backup_select_ms / args.steps
        out.pop("nn_in_loop", None)
        out.pop("tree_kernels", None)
    if rank == 0:
        # the dominant kernel's roofline, on one stream (single_stream_leg): per-launch HIP events
        leg = single_stream_leg(args, cfg, local, cfg["precision"])
        lp = leg["positions"]
        nn_blob = float(_abi.load().oaz_nn_device_bytes(cfg["blocks"], getattr(_abi, PREC_ABI[cfg["precision"]])))
        out["roofline"] = {
            "bound": "mfma", "kernel": NN_KERNEL[cfg["precision"]],
            "achieved": leg["achieved"], "peak": PEAK_TFLOPS[cfg["precision"]], "unit": "TFLOP/s",
            "frac": leg["achieved"] / PEAK_TFLOPS[cfg["precision"]],
            "traffic": (traffic or {}).get("bytes_per_sim_step"),
            "measured_on": "the same workload on one stream (oaz_config.parts = 1; 2 warm-up + 2 timed plies, no "
                           "staggered starts), HIP events around the NN launches of every 8th simulation step; "
                           "rocprofv3 kernel trace of the same launches: tools/trace_steady.py (last dispatches)",
            "flop_per_launch": leg["flops"], "avg_launch_ms": leg["avg_launch_ms"], "launches": leg["launches"],
            "positions_per_launch": lp, "flop_accounting": "SURVEY 8d dense MACs x2 per sim",
            "achieved_nonzero": leg["nonzero_achieved"],
            "frac_nonzero": leg["nonzero_achieved"] / PEAK_TFLOPS[cfg["precision"]],
            # per launch: the packed weight image into each XCD's L2 (a launch starts with cold L2s:
            # profiles/r05_nn_l2_standalone_pmc.txt) + 24 B state in + 204 B policy / value out per position
            "algorithmic_bytes_per_launch": XCDS * nn_blob + lp * (24 + 204),
            "algorithmic_note": f"weights {nn_blob / 1e6:.3f} MB x {XCDS} XCD L2 fills per launch (the L2s do not keep "
                                "them across launches; the Infinity Cache serves the fills) + 24 B state in + 204 B "
                                "policy / value out per position; per simulation step the launches of every game part",
            "algorithmic_bytes_single_weight_copy": nn_blob + lp * (24 + 204),
            # what `traffic` measures: one simulation step of the timed loop = one launch per game part
            "algorithmic_bytes_per_sim_step": (traffic or {}).get("game_parts", 1) * XCDS * nn_blob
                                              + cfg["games"] * (24 + 204),
            # the SURVEY 8d formula itself: ONE copy of the weight image per simulation step
            "algorithmic_bytes_per_sim_step_single_copy": nn_blob + cfg["games"] * (24 + 204),
            "traffic_detail": traffic,
            "peak_note": {"fp32": "F32 MFMA dense peak", "bf16": "BF16 dense MFMA peak",
                          "fp32_split": "BF16 dense MFMA peak / 6 products per fp32 MAC",
                          "fp32_split16": "FP16 dense MFMA peak / 3 products per fp32 MAC"}[cfg["precision"]],
            "frac_of_fp32_mfma_peak": leg["achieved"] / PEAK_TFLOPS["fp32"]}
        rf = out["roofline"]
        if rf["traffic"]:
            # measured HBM bytes per simulation step against the single-copy formula (the weights read once,
            # SURVEY 8d) and against the same formula plus the per-launch refill of every XCD's L2
            rf["traffic_vs_single_copy"] = rf["traffic"] / rf["algorithmic_bytes_per_sim_step_single_copy"]
            rf["traffic_vs_with_xcd_refills"] = rf["traffic"] / rf["algorithmic_bytes_per_sim_step"]
            rf["traffic_note"] = ("traffic / the single-copy formula: the excess is the weight image re-read into "
                                  f"each of the {XCDS} XCD L2s on every launch (kernel boundaries invalidate the "
                                  "L2s; profiles/r05_nn_l2_standalone_pmc.txt), a per-launch refill overhead, not "
                                  "algorithmic bytes")
        if clock:
            # the clock of the measured launches: the kernel's cycles per launch (PMC pass) over the
            # un-profiled HIP-event launch time above; the peak scaled to that clock (2400 MHz nominal)
            mhz = clock["cycles_per_launch"] / (leg["avg_launch_ms"] * 1e-3) / 1e6
            out["roofline"].update(
                sclk_mhz=mhz, peak_at_measured_clock=PEAK_TFLOPS[cfg["precision"]] * mhz / NOMINAL_MHZ,
                frac_at_measured_clock=out["roofline"]["frac"] * NOMINAL_MHZ / mhz,
                frac_nonzero_at_measured_clock=out["roofline"]["frac_nonzero"] * NOMINAL_MHZ / mhz,
                rocprof_avg_launch_ms=clock["profiled_avg_launch_ms"], clock_detail=clock,
                clock_note="sclk = GRBM_GUI_ACTIVE/8 cycles per k_nn_ launch (rocprofv3 pass on this box, one stream) "
                           "/ the HIP-event launch time above; rocprof_avg_launch_ms = the same pass's kernel-trace "
                           "duration of those launches (profiled launches run at profiled_clock_mhz)")
        if grp_mode:  # the timed region's own dominant kernel (k_search_grp); the NN kernel's leg stays beside it
            sk = out["search_kernel"]
            nn_leg = dict(out["roofline"])
            out["roofline"] = {
                "bound": "mfma", "kernel": sk["kernel"], "achieved": sk["achieved_TFLOPs"],
                "peak": PEAK_TFLOPS[cfg["precision"]], "unit": "TFLOP/s",
                "frac": sk["achieved_TFLOPs"] / PEAK_TFLOPS[cfg["precision"]],
                "traffic": (traffic or {}).get("bytes_per_launch"),
                "flop_per_launch": FLOP_PER_SIM[cfg["blocks"]] * sk["sims_per_launch"],
                "avg_launch_ms": sk["avg_launch_ms"], "launches": sk["launches"],
                "measured_on": "the timed region: HIP events around every k_search_grp launch (each covers "
                               "one root-noise chunk, a whole C2 ply, of every game, tree work included)",
                "flop_accounting": "SURVEY 8d dense MACs x2 per sim", "nn_kernel_single_stream": nn_leg,
                # per simulation: the network's state in and policy / value out (24 + 204 B), the tree work
                # (~1.95 KB at C3 depth and branching), the weights once per 16-game workgroup
                "algorithmic_bytes_per_launch": sk["sims_per_launch"] * (24 + 204 + 1954)
                                                + 0.96e6 * (cfg["games"] + 15) // 16 / 256,
                "traffic_detail": traffic if (traffic or {}).get("kernel") == "k_search_grp" else None}
            tr = out["roofline"]["traffic_detail"]
            if tr:  # FETCH_SIZE x1 .. x2 (the tree records are scattered, the weight reads streams)
                alg = out["roofline"]["algorithmic_bytes_per_launch"]
                out["roofline"]["traffic_vs_algorithmic"] = [tr["bytes_per_launch_raw"] / alg,
                                                             tr["bytes_per_launch"] / alg]
        bs = (out.get("tree_kernels") or {}).get("backup_select") or {}
        sq = (bs.get("pmc") or {}).get("sq")
        if leg.get("tree_launch_us"):
            bs["single_stream_launch_us"] = leg["tree_launch_us"]  # all games in one launch, nothing beside it
            if sq:
                mhz = out["roofline"].get("sclk_mhz") or NOMINAL_MHZ
                parts = max(1, (traffic or {}).get("game_parts", 1))
                floor_us = sq["valu_cycles_per_simd_per_launch"] * parts / mhz
                sq["valu_floor_frac_single_stream"] = floor_us / leg["tree_launch_us"]
                sq["clock_mhz_used"] = mhz
        if world == 1 and not args.no_exact:
            out["leaf_compaction"] = compaction_leg(args, cfg, local, stagger)
        if not args.no_exact and world == 1 and cfg["precision"] in ("fp32_split16", "fp32_split"):
            out["exact_fp32"] = exact_fp32_leg(args, cfg, local)
        if not args.no_cpu_baseline and world == 1:
            try:  # after the timed region: a baseline failure must not lose the measured line
                out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds, args.cpu_threads)
            except Exception as ex:  # noqa: BLE001
                print(f"bench: cpu_baseline failed: {ex!r}", file=sys.stderr, flush=True)
                out["cpu_baseline"] = {"error": repr(ex)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not checks["ok"]:
        print(f"bench: invalid run: {checks}", file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
