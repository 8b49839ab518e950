"""bench.py - images/sec of the YOLO-SOD inference step on MI355X (BASELINE.json metric), one process per GPU.

step = one predictor pass over one batch of synthetic 640x640 images already resident in HBM:
       backbone/neck convs (PyTorch-ROCm) + HIP MAFN operators + HIP Detect decode + HIP batched NMS
       (+ for N > 1 the RCCL all-gather of the padded detections: the path's single exchange step).
Weak scaling: every rank processes its own batch of 32 images; value = N * 32 * K / max-over-ranks(time of K steps).

Usage: python bench.py [--gpus N --steps K --warmup W]; for N > 1 launch with
       python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
              bench.py --gpus N --steps K --warmup W
       `python bench.py --gpus N` with no WORLD_SIZE in the environment starts those N ranks itself: the parent
       (which makes no GPU call) runs torch.distributed.run as a child process and exits with its code (the
       reference's DDP entry does the same, ultralytics/engine/trainer.py:197-200, utils/dist.py:56-66).
Rank 0 prints ONE compact JSON line (< 4 KB): the contract fields, `roofline` of the dominant HIP operator (measured
live with HIP events inside the timed region), `path_roofline`, `cpu_baseline` (the oracle CPU model timed on the
host cores, rank 0 at N = 1 only) and, at N = 1, `configs`: BASELINE configs[3] (n1280, bs 8) and configs[4] (m640
bf16, bs 64), each timed in its own region of the same process (value, ms_per_step, roofline / path fractions).
Every per-operator figure (hip_ops, backbone_hip_ops, the full cpu_baseline) goes to the --detail-json file, which
scripts/roofline_from_csv.py checks against --ops-csv. Roofline fractions are quoted against the ceiling of the
arithmetic each kernel issues (perf.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
# MIOpen solver choices for the backbone / neck convs: a user find-db recorded on MI355X with MIOPEN_FIND_MODE=NORMAL
# (every applicable solver timed; scripts/miopen_db.sh), so every run takes the same solvers instead of whatever the
# first-call search of its box measured (round 3: one fresh box chose Winograd f3x2 over the implicit GEMM for the
# stride-2 convs, 18.0 vs 16.4 ms per step). Set MIOPEN_USER_DB_PATH to override.
os.environ.setdefault("MIOPEN_USER_DB_PATH", str(ROOT / "yolo-sod_amd" / "miopen_db"))
import yolosod_import  # noqa: E402,F401

from yolosod_amd import _hip, perf  # noqa: E402
from yolosod_amd.engine.predictor import (DetectionPredictor, seeded_images, shard_bounds,  # noqa: E402
                                          sharded_predict)
from yolosod_amd.nn.tasks import build_model  # noqa: E402

METRIC = "images/sec @640×640 bs=32, 1→8 MI355X; mAP@0.5:0.95 parity vs CPU ref"
CONFIGS = {
    # name: (yaml, imgsz, batch per GPU, label, dtype) - BASELINE.json configs[1..4]; n640 is the metric's workload
    "n640": ("yolov12-sod-fusion-v5-simple.yaml", 640, 32, "yolov12n-sod (paper YAML)", torch.float32),
    "n1280": ("yolov12-sod-fusion-v5-simple.yaml", 1280, 8, "yolov12n-sod (paper YAML)", torch.float32),
    # configs[4]: bf16 model (parameters + activations bf16, fp32 accumulation; decode / NMS fp32), DESIGN.md 9
    "m640": ("yolov12m-sod.yaml", 640, 64, "yolov12m-sod (paper graph at v12 m scale)", torch.bfloat16),
    "m640f32": ("yolov12m-sod.yaml", 640, 64, "yolov12m-sod (paper graph at v12 m scale)", torch.float32),
}
DTYPE_NAME = {torch.float32: "f32", torch.bfloat16: "bf16"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpu():
    """(cpu model string, cores usable by this process): physical cores within the affinity mask, capped by a
    cgroup CPU quota when one is set."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    allowed = len(os.sched_getaffinity(0))
    try:
        import psutil
        per_core = max(1, (psutil.cpu_count() or allowed) // max(1, psutil.cpu_count(logical=False) or allowed))
    except Exception:
        per_core = 1
    cores = max(1, allowed // per_core)
    for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            q = open(f).read().split()
            if q[0] not in ("max", "-1"):
                period = int(q[1]) if len(q) > 1 else int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
                cores = max(1, min(cores, int(q[0]) // period))
            break
        except (OSError, ValueError, IndexError):
            continue
    return model, cores


def _median(v):
    v = sorted(v)
    return v[len(v) // 2] if len(v) % 2 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2])


def cpu_baseline(cfg_yaml, imgsz, warmup=2, iters=5, batch_all=8, single=True):
    """the oracle CPU model (fp32 PyTorch-CPU restatement + C NMS, pinned to the reference
    by tests/golden) on this host's cores. All usable physical cores on a bounded sample of the workload
    (``batch_all`` images of the same 640x640 batch per iteration) and 1 thread on BASELINE configs[0] (one
    640x640 image: the reference's default, OMP_NUM_THREADS=1 at ultralytics/__init__.py:8-9); ``warmup``
    untimed + the median of ``iters`` timed iterations each. The MAFN + decode + NMS share is timed with hooks
    on the operator modules inside the same iterations; NMS alone on loaded synthetic tensors (1k/10k/30k
    candidates per image)."""
    from oracle.model_ref import build_cpu_model
    from oracle.nms import non_max_suppression_ref
    from yolosod_amd.nn import modules as M
    model_name, cores = host_cpu()
    m = build_cpu_model(cfg_yaml)
    hot_t = []
    t_in = {}

    def pre(mod, inp):
        t_in[id(mod)] = time.perf_counter()

    def post(mod, inp, out):
        hot_t.append(time.perf_counter() - t_in.pop(id(mod)))

    hot = (M.SE, M.CBAM_Block, M.CA_Block, M.A2_Attn, M.SwinBlock, M.MambaBlock)
    for mod in m.modules():
        if isinstance(mod, hot):
            mod.register_forward_pre_hook(pre)
            mod.register_forward_hook(post)
    det = m.model[-1]
    inf = det._inference

    def timed_inference(x):  # decode (Detect._inference, head.py:100-131)
        t0 = time.perf_counter()
        y = inf(x)
        hot_t.append(time.perf_counter() - t0)
        return y

    det._inference = timed_inference

    def run(threads, bs):
        torch.set_num_threads(threads)
        x = seeded_images(0, bs, imgsz)
        tot, hotv = [], []
        with torch.inference_mode():
            for it in range(warmup + iters):
                hot_t.clear()
                t0 = time.perf_counter()
                y = m(x)[0]
                t1 = time.perf_counter()
                non_max_suppression_ref(y.numpy().copy(), 0.25, 0.7, max_det=300)
                t2 = time.perf_counter()
                if it >= warmup:
                    tot.append(t2 - t0)
                    hotv.append(sum(hot_t) + (t2 - t1))
        med = _median(tot)
        return {"threads": threads, "batch": bs, "value": round(bs / med, 3), "unit": "images/s",
                "ms_per_image": round(med / bs * 1e3, 2),
                "mafn_decode_nms_ms_per_image": round(_median(hotv) / bs * 1e3, 2),
                "iterations": f"{warmup} warm-up + median of {iters}"}

    t_start = time.perf_counter()
    all_cores = run(cores, batch_all)
    one = run(1, 1) if single else None
    # NMS alone, loaded: oracle NMS per image on the same synthetic tensors bench.py times on the GPU
    nms = {}
    for n_cand in NMS_LOADS:
        pred = loaded_predictions(2, 34000, 10, n_cand, 50, 0.25, 0, torch.device("cpu")).numpy()
        ts = []
        for b in range(pred.shape[0]):
            t0 = time.perf_counter()
            non_max_suppression_ref(pred[b:b + 1].copy(), 0.25, 0.7, max_det=300)
            ts.append(time.perf_counter() - t0)
        nms[str(n_cand)] = round(_median(ts) * 1e3, 2)
    det._inference = inf
    return {"value": all_cores["value"], "unit": "images/s", "cores": cores, "kind": "port",
            "cpu_model": model_name,
            "sample": f"{batch_all} of the {imgsz}x{imgsz} images per iteration, forward + decode + NMS "
                      f"(conf 0.25), oracle fp32 CPU model, torch threads={cores} (usable physical cores), "
                      f"{warmup} warm-up + median of {iters}; total CPU wall {time.perf_counter() - t_start:.1f}s",
            "all_cores": all_cores,
            "single_thread_configs0": one,
            "nms_loaded_ms_per_image": nms}


NMS_LOADS = (1000, 10000, 30000)


def loaded_predictions(B, A, nc, n_cand, clusters, conf, seed, dev, img=640.0):
    """Synthetic Detect output [B, 4+nc, A] with exactly n_cand anchors per image scoring above ``conf`` (a main
    class score in (conf, 1)), boxes (xywh) drawn around ``clusters`` centres with heavy overlap, as trained heads
    produce. Random-init weights leave NMS empty (nothing clears conf 0.25), so NMS at load is timed on these."""
    g = torch.Generator(device=dev).manual_seed(seed)
    k = torch.randint(0, clusters, (B, A), generator=g, device=dev)
    cen = torch.rand(B, clusters, 4, generator=g, device=dev)
    cx, cy = cen[..., 0] * img, cen[..., 1] * img
    cw, ch = 8 + cen[..., 2] * 112, 8 + cen[..., 3] * 112
    jit = torch.randn(4, B, A, generator=g, device=dev) * 0.08
    gat = lambda t: torch.gather(t, 1, k)  # noqa: E731
    w, h = gat(cw), gat(ch)
    box = torch.stack([gat(cx) + jit[0] * w, gat(cy) + jit[1] * h, w * jit[2].exp(), h * jit[3].exp()], 1)
    cls = torch.rand(B, nc, A, generator=g, device=dev) * conf * 0.9
    sel = torch.rand(B, A, generator=g, device=dev).argsort(1)[:, :n_cand]
    main = torch.randint(0, nc, (B, n_cand), generator=g, device=dev)
    val = conf + (1 - conf) * torch.rand(B, n_cand, generator=g, device=dev)
    cls[torch.arange(B, device=dev)[:, None], main, sel] = val
    return torch.cat([box, cls], 1).contiguous()


def nms_loaded(dev, B=32, A=34000, nc=10, reps=10):
    """HIP NMS (predict mode: conf 0.25, iou 0.7, max_det 300) on [B, 4+nc, A] tensors with 1k / 10k / 30k
    candidates per image, HIP events around each call (fresh copy per call: NMS rewrites boxes in place)."""
    from yolosod_amd.utils.ops import non_max_suppression_padded
    res = {}
    for n_cand in NMS_LOADS:
        pred = loaded_predictions(B, A, nc, n_cand, 50, 0.25, 0, dev)
        work = [pred.clone() for _ in range(reps + 3)]
        ms = []
        for i, w in enumerate(work):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _, counts, _ = non_max_suppression_padded(w, 0.25, 0.7, max_det=300)
            e1.record()
            if i >= 3:
                ms.append((e0, e1))
        torch.cuda.synchronize()
        t = sorted(a.elapsed_time(b) for a, b in ms)
        res[str(n_cand)] = {"ms_per_call": round(t[len(t) // 2], 4), "images": B,
                            "kept_per_image": round(float(counts.float().mean()), 1)}
    return res


def load_traffic():
    p = ROOT / "profiles" / "traffic.json"
    if p.exists():
        try:
            return json.loads(p.read_text())
        except Exception:
            return None
    return None


def measure(name, world, rank, dev, steps, warmup, conf, ops_csv=None, time_all=False):
    """One config: warmup, K timed steps (barrier + synchronize on both sides, max over ranks), per-operator HIP
    event timings -> rooflines. Returns (result dict, predictor)."""
    cfg_yaml, imgsz, bs, label, dtype = CONFIGS[name]
    dname = DTYPE_NAME[dtype]
    model = build_model(cfg_yaml, seed=0, device=dev, dtype=dtype)
    predictor = DetectionPredictor(model, conf=conf, iou=0.7, max_det=300)
    # one global seeded batch of world * bs images (image i from seed 1000 + i); each rank holds its shard, resident
    # in HBM in the model's dtype before the timed region (the predictor's .to(dtype) is then a no-op)
    n_global = world * bs
    lo, hi = shard_bounds(n_global, rank, world)
    x = seeded_images(lo, hi, imgsz, device=dev).to(dtype)

    def step():
        # the timed step is the same at every N: no host sync inside it. The split-range guard's flag word is read
        # once after the timed region on every rank (split_range_flagged below), not per step
        if world > 1:  # shard -> rank-local predict -> all-gather of the padded detections + kept indices
            return sharded_predict(predictor.predict_padded, n_global, lambda a, b: x, split_guard=False)[1]
        return predictor.predict_padded(x)[1]

    # HIP events bracket only the hot-path operators and what is billed to them (perf.PathSelect; --time-all-ops:
    # every launch); the last warmup step runs through the filter so that it knows the plain variants to time
    select = None if time_all else perf.PathSelect()
    t_w = time.perf_counter()
    # with --warmup 0 one untimed primer step still runs through the filter (it learns the plain variants there)
    for i in range(max(warmup, 1 if select is not None else 0)):
        if i == max(warmup, 1) - 1 and select is not None:
            with _hip.op_timer(select):
                step()
        else:
            step()
    torch.cuda.synchronize()
    log(f"[rank {rank}] {name}: warmup {warmup} steps {time.perf_counter() - t_w:.2f}s")

    def timed():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        with _hip.op_timer(select) as timer:
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t1 = time.perf_counter()
        # one read of the split-range flag per rank after the region (fp32 configs; bf16 runs no split kernels)
        flagged = float(dtype == torch.float32 and _hip.split_range_flag(reset=True, device=dev))
        red = torch.tensor([t1 - t0, flagged], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(red, op=dist.ReduceOp.MAX)
        return float(red[0].item()), bool(red[1].item()), timer

    elapsed, flagged, timer = timed()
    redone = False
    if flagged:
        # an operand left the fp16-split kernels' range inside the region: the predictor would redo such a batch on
        # the exact fp32 kernels, so the line reports the region timed that way instead of the flagged steps
        log(f"[rank {rank}] {name}: split-range flag set in the timed region; re-timing on the exact fp32 kernels")
        with _hip.exact_fp32_matrix():
            elapsed, _, timer = timed()
        redone = True
    durs = timer.durations_ms()

    # per-operator live timings (HIP events on the launch stream) -> roofline of the dominant operator; the
    # producer billing uses the same region's launches only (perf.producer_billing)
    if ops_csv is not None:
        ops_csv.extend(perf.calls_to_rows(name, steps, durs))
    ops, backbone, path_roofline = perf.summarize(durs, steps)
    dom = ops[0]
    bound = dom["bound"]
    if bound == "mfma":
        achieved, peak, unit = dom["TFLOPs"], perf.method_peak_tflops(dom["key"]), "TFLOP/s"
    else:
        achieved, peak, unit = dom["GBps"], perf.PEAK_HBM_GBS, "GB/s"
    traffic = load_traffic()
    roofline = {"bound": bound, "achieved": achieved, "peak": round(peak, 1), "unit": unit,
                "frac": round(achieved / peak, 4),
                "traffic": (traffic or {}).get(f"{dom['op']}:{'x'.join(map(str, dom['shape']))}"),
                "kernel": f"{dom['op']}{tuple(dom['shape'])} (one C-ABI call = its launch sequence)",
                "algorithmic_per_launch": dom["flops"] if bound == "mfma" else dom["bytes"],
                "peak_basis": ("matrix-core ceiling of the method the kernel computes with" if bound == "mfma"
                               else "HBM3E spec")}
    if bound == "mfma":
        dpeak = perf.peak_tflops(dom["key"])
        if abs(dpeak - peak) > 1e-6:
            # the fp32 Swin / A2 / head kernels run each fp32 product as 3 exact fp16 products of two-term splits
            # (csrc/swin_x3.hip): their roof is the fp16 peak / 3; the fp32 MFMA peak is kept as a secondary figure
            roofline["method"] = "fp16 two-term splits on v_mfma_f32_16x16x32_f16, 3 products per fp32 product"
        roofline["frac_vs_dtype_peak"] = round(achieved / dpeak, 4)
        roofline["dtype_peak"] = dpeak

    t_meas = path_roofline["t_meas_ms"]
    value = world * bs * steps / elapsed
    res = {"value": round(value, 2), "unit": "images/s", "ms_per_step": round(elapsed / steps * 1e3, 3),
           "steps": steps, "warmup": warmup, "dtype": dname,
           "data": f"synthetic: torch.rand images in HBM, seed-0 random-init weights of {label}",
           "config": {"name": name, "workload": f"{label} {imgsz}x{imgsz}, {bs} images per GPU, fused {dname} "
                                  f"forward + decode + NMS(conf={conf}, iou=0.7)",
                      "imgsz": imgsz, "batch_per_gpu": bs, "global_batch": bs * world, "parallelism": f"dp{world}"},
           "roofline": roofline, "path_roofline": path_roofline, "split_range_flagged": flagged,
           "split_range_redone_exact": redone,
           "hip_ops_ms_per_step": round(t_meas, 3),
           "hip_ops": [{k: v for k, v in o.items() if k not in ("bytes", "flops", "key")} for o in ops],
           "backbone_hip_ms_per_step": round(sum(o["total_ms_per_step"] for o in backbone), 3),
           "backbone_hip_ops": backbone[:12]}
    return res, predictor, cfg_yaml, imgsz


# BASELINE.json configs[3] / configs[4] on one GPU, timed in the same process after the headline (N = 1 only)
EXTRA_CONFIGS = ("m640", "n1280")
LINE_LIMIT = 4000  # bytes: the driver parses the last stdout line; round 4's 20 KB line did not parse


def _op_name(o):
    return f"{o['op']}:{'x'.join(map(str, o['shape']))}"


def _compact_roofline(r):
    keep = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "algorithmic_per_launch",
            "frac_vs_dtype_peak")
    out = {k: r[k] for k in keep if k in r}
    out["kernel"] = out.get("kernel", "").split(" (")[0]
    return out


def compact_line(result, detail_path=None):
    """The one stdout JSON line from the full result: contract fields, roofline (+traffic), path_roofline, the
    cpu_baseline summary, NMS-at-load per call, per-op ms of the headline and per extra config only value /
    ms_per_step / roofline.frac / path_roofline.frac. Everything else stays in the detail file."""
    head = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "split_range_flagged", "hip_ops_ms_per_step",
            "backbone_hip_ms_per_step")
    line = {k: result[k] for k in head if k in result}
    line["roofline"] = _compact_roofline(result["roofline"])
    pr = result["path_roofline"]
    line["path_roofline"] = {k: pr[k] for k in ("t_min_ms", "t_meas_ms", "frac", "frac_vs_dtype_peak")}
    if "mafn" in pr:  # SURVEY 8(d)'s fixed path: MAFN + decode + NMS only (perf.mafn_path)
        line["mafn_path"] = {k: pr["mafn"][k] for k in ("t_hbm_floor_ms", "t_min_ms", "t_meas_ms", "frac",
                                                         "frac_vs_hbm_floor")}
    line["hip_ops_avg_ms"] = {_op_name(o): o["avg_ms"] for o in result.get("hip_ops", [])}
    nl = result.get("nms_loaded")
    line["nms_loaded_ms_per_call"] = None if nl is None else {k: v["ms_per_call"] for k, v in nl.items()}
    cb = result.get("cpu_baseline")
    if cb is not None and "error" not in cb:
        one = cb.get("single_thread_configs0") or {}
        cb = {"value": cb["value"], "unit": cb["unit"], "cores": cb["cores"], "kind": cb["kind"],
              "sample": cb["sample"], "cpu_model": cb.get("cpu_model"),
              "mafn_decode_nms_ms_per_image": (cb.get("all_cores") or {}).get("mafn_decode_nms_ms_per_image"),
              "single_thread_configs0_value": one.get("value"),
              "nms_loaded_ms_per_image": cb.get("nms_loaded_ms_per_image")}
    line["cpu_baseline"] = cb
    if "configs" in result:
        line["configs"] = {n: {"value": c["value"], "ms_per_step": c["ms_per_step"], "dtype": c["dtype"],
                               "batch_per_gpu": c["config"]["batch_per_gpu"], "imgsz": c["config"]["imgsz"],
                               "roofline_frac": c["roofline"]["frac"], "roofline_kernel":
                                   c["roofline"]["kernel"].split(" (")[0],
                               "path_roofline_frac": c["path_roofline"]["frac"],
                               "mafn_path_frac": (c["path_roofline"].get("mafn") or {}).get("frac")}
                           for n, c in result["configs"].items()}
    if detail_path:
        line["detail"] = str(detail_path)
    txt = json.dumps(line)
    if len(txt.encode()) > LINE_LIMIT:  # never exceed: drop the per-op map first, then the NMS / CPU extras
        for k in ("hip_ops_avg_ms", "nms_loaded_ms_per_call"):
            line.pop(k, None)
            txt = json.dumps(line)
            if len(txt.encode()) <= LINE_LIMIT:
                break
    return line


def launcher_cmd(argv, gpus, port):
    """Child command that starts ``gpus`` ranks of this script (one process per GPU, RCCL), as the driver does."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *argv]


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="n640", choices=list(CONFIGS))
    ap.add_argument("--conf", type=float, default=0.25)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-nms-load", action="store_true")
    ap.add_argument("--no-extra-configs", action="store_true", help="skip the m640 / n1280 blocks (N = 1 only)")
    ap.add_argument("--time-all-ops", action="store_true",
                    help="HIP events around every library launch in the timed region (default: the hot-path operators "
                         "and the producers billed to them only; the events cost the step a few per cent)")
    ap.add_argument("--miopen-benchmark", action="store_true", help="torch.backends.cudnn.benchmark (MIOpen find)")
    ap.add_argument("--ops-csv", default=None,
                    help="write every timed C-ABI launch (HIP event ms, rank 0) of every config to this CSV: "
                         "scripts/roofline_from_csv.py recomputes hip_ops / producer billing / path_roofline from it")
    ap.add_argument("--detail-json", default=str(ROOT / "gpurun_out" / "bench_detail.json"),
                    help="full result (every hip_ops / backbone_hip_ops entry, the full cpu_baseline) as one JSON "
                         "file; '' to skip")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher around us: start the N ranks as a child process (this process has made no GPU call) and pass
        # its exit code on; rank 0 of the child prints the line
        import subprocess
        cmd = launcher_cmd(sys.argv[1:], args.gpus, _free_port())
        log("launching: " + " ".join(cmd))
        env = dict(os.environ, MASTER_ADDR="127.0.0.1")
        sys.exit(subprocess.run(cmd, env=env).returncode)

    if args.miopen_benchmark:
        torch.backends.cudnn.benchmark = True
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    rows = [] if args.ops_csv and rank == 0 else None
    head, predictor, cfg_yaml, imgsz = measure(args.config, world, rank, dev, args.steps, args.warmup, args.conf,
                                               ops_csv=rows, time_all=args.time_all_ops)
    result = {"metric": METRIC, "value": head["value"], "unit": "images/s", "n_gpus": world, "steps": args.steps,
              "warmup": args.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
              "scaling": "weak", "vs_baseline": None}
    result.update({k: v for k, v in head.items() if k not in result})
    result["nms_loaded"] = None
    result["cpu_baseline"] = None
    if not args.no_nms_load:  # after the timed region, same process: NMS at controlled candidate loads
        result["nms_loaded"] = nms_loaded(dev)
    del predictor
    torch.cuda.empty_cache()
    if world == 1 and args.config == "n640" and not args.no_extra_configs:
        # configs[3] (n1280 bs 8) and configs[4] (m640 bf16 bs 64): their own timed regions, same contract
        result["configs"] = {}
        for name in EXTRA_CONFIGS:
            sub, pred, _, _ = measure(name, 1, 0, dev, args.steps, args.warmup, args.conf, ops_csv=rows,
                                      time_all=args.time_all_ops)
            result["configs"][name] = sub
            del pred
            torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            # m scale: ~4x the n model's CPU work per image - a smaller sample keeps the same ~10-30 s budget
            m_scale = cfg_yaml.startswith("yolov12m")
            result["cpu_baseline"] = cpu_baseline(cfg_yaml, imgsz, batch_all=2 if m_scale else 8,
                                                  single=not m_scale)
        except Exception as e:  # report, never hide
            result["cpu_baseline"] = {"error": repr(e)}
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rows is not None:
        import csv
        with open(args.ops_csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=perf.CSV_FIELDS)
            w.writeheader()
            w.writerows(rows)
    if rank == 0:
        detail = None
        if args.detail_json:
            try:
                Path(args.detail_json).parent.mkdir(parents=True, exist_ok=True)
                Path(args.detail_json).write_text(json.dumps(result) + "\n")
                dp = Path(args.detail_json).resolve()
                detail = str(dp.relative_to(ROOT)) if dp.is_relative_to(ROOT) else str(dp)
            except OSError as e:
                log(f"detail json not written: {e!r}")
        print(json.dumps(compact_line(result, detail)), flush=True)


if __name__ == "__main__":
    main()
