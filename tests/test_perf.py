"""perf.summarize: the hip_ops / producer billing / path roofline bench.py reports, recomputed from per-launch rows
(CPU only; the numbers are synthetic)."""
import pytest

import yolosod_import  # noqa: F401
from yolosod_amd import perf

CAP = ("bias_act", (32, 128, 80, 80), "capool")
PLAIN = ("bias_act", (32, 128, 80, 80), None)
PLAIN_RES = ("bias_act", (32, 128, 80, 80), "res")
CA = ("ca", (32, 128, 80, 80), 8)
SE_PROD = ("bias_act", (32, 32, 320, 320), "sum")
SE = ("se", (32, 32, 320, 320), 8)
THIN = ("conv1x1_thin", (32, 96, 160, 160), (64, "summax"))
THIN_PLAIN = ("conv1x1_thin", (32, 96, 160, 160), (64, False, False))
CBAM = ("cbam", (32, 64, 160, 160), 4)


def _calls():
    return [(CAP, 0.13), (PLAIN, 0.06), (PLAIN, 0.065), (PLAIN_RES, 0.5), (CA, 0.08),
            (SE_PROD, 0.15), (SE, 0.17), (THIN, 0.19), (THIN_PLAIN, 0.16), (CBAM, 0.13)]


def _by_op(ops):
    return {(o["op"], tuple(o["shape"])): o for o in ops}


def test_producer_billed_from_the_same_region():
    ops, backbone, path = perf.summarize(_calls(), steps=1)
    o = _by_op(ops)
    # CA: in-model capool minus the mean of the in-model plain launches without a residual (the "res" one excluded)
    assert o[("ca", CA[1])]["producer_extra_ms"] == pytest.approx(0.13 - 0.0625, abs=1e-4)
    assert o[("ca", CA[1])]["avg_ms"] == pytest.approx(0.08 + 0.0675, abs=1e-4)
    # CBAM on the thin conv: stats variant minus the plain variant of the same shape and Cout
    assert o[("cbam", CBAM[1])]["producer_extra_ms"] == pytest.approx(0.03, abs=1e-4)
    # SE: no plain variant of that shape in the region -> plain pass priced at the HBM roof (upper bound)
    roof = 2 * 32 * 32 * 320 * 320 * 4 / 8e12 * 1e3
    assert o[("se", SE[1])]["producer_extra_ms"] == pytest.approx(0.15 - roof, abs=1e-4)
    assert "HBM roof" in o[("se", SE[1])]["producer"]
    assert {b["op"] for b in backbone} == {"bias_act", "conv1x1_thin"}
    t_meas = sum(x["total_ms_per_step"] for x in ops)
    assert path["t_meas_ms"] == pytest.approx(t_meas, abs=1e-3)
    assert path["frac"] == pytest.approx(path["t_min_ms"] / path["t_meas_ms"], abs=1e-3)


def test_csv_rows_round_trip_keys_exactly():
    calls = _calls() + [(("bias_act", (8, 64, 40, 40), "summax+res", 2), 0.02), (("cbam", (8, 64, 40, 40), 4, 2), 0.03),
                        (("swin", (32, 64, 160, 160), (2, 7, 256)), 0.5), (("nms", (32, 10, 34000), 300), 0.03)]
    rows = perf.calls_to_rows("n640", 10, calls)
    assert [r["seq"] for r in rows] == list(range(len(calls)))
    assert perf.rows_to_calls(rows) == calls
    a = perf.summarize(calls, 10)
    b = perf.summarize(perf.rows_to_calls(rows), 10)
    assert [(o["op"], o["avg_ms"], o.get("producer_extra_ms")) for o in a[0]] == \
        [(o["op"], o["avg_ms"], o.get("producer_extra_ms")) for o in b[0]]


def test_bf16_residual_producer_pairs_with_its_plain_residual_variant():
    prod = ("bias_act", (8, 64, 40, 40), "summax+res", 2)
    plain = ("bias_act", (8, 64, 40, 40), "res", 2)
    gate, gshape, pkey, nbytes = perf.producer_of(prod)
    assert (gate, gshape, pkey) == ("cbam", (8, 64, 40, 40), plain)
    assert nbytes == 3 * 8 * 64 * 40 * 40 * 2
    billed = perf.producer_billing(perf.aggregate([(prod, 0.05), (plain, 0.04), (plain, 0.02)]))
    assert billed[("cbam", (8, 64, 40, 40))][0] == pytest.approx(0.02)


def test_fused_gate_conv_bills_the_gate_and_the_producer():
    """A gate fused into its consumer conv (nn/tasks.py GATE_FUSE): the gate-only launches and the producer's extra
    time go to the fused operator "<gate>_conv", whose cost counts x read once, the conv output written once and
    the conv FLOPs at the fp16-split ceiling."""
    gate = ("se_gate", (32, 32, 320, 320), 8)
    fused = ("se_conv", (32, 32, 320, 320), (64, 8))
    calls = [(SE_PROD, 0.15), (gate, 0.005), (fused, 0.14), (SE_PROD, 0.15), (gate, 0.005), (fused, 0.14)]
    ops, backbone, path = perf.summarize(calls, steps=2)
    o = _by_op(ops)
    assert ("se_gate", (32, 32, 320, 320)) not in o and [b["op"] for b in backbone] == ["bias_act"]
    f = o[("se_conv", (32, 32, 320, 320))]
    extra = 0.15 - 32 * 32 * 320 * 320 * 4 * 2 / 8e12 * 1e3  # producer vs its plain pass at the HBM roof
    assert f["launches"] == 2 and f["avg_ms"] == pytest.approx(0.145 + extra, abs=1e-4)
    nbytes, flops = perf.op_cost(fused)
    assert nbytes >= (32 * 32 * 320 * 320 + 32 * 64 * 160 * 160) * 4
    assert flops >= 2 * 32 * 160 * 160 * 64 * 32 * 9
    assert perf.method_peak_tflops(fused) == pytest.approx(perf.PEAK_BF16_MFMA_TFLOPS / 3)
    assert path["t_meas_ms"] == pytest.approx(f["avg_ms"], abs=1e-3)


def test_path_select_times_the_path_its_producers_and_their_plain_variants_only():
    """bench.py's timed region brackets only these launches with HIP events (perf.PathSelect)."""
    sel = perf.PathSelect()
    plain = ("bias_act", (32, 128, 80, 80), None)
    assert not sel(plain)  # before its producer was seen: a plain backbone epilogue
    assert sel(("swin", (32, 64, 160, 160), (2, 7, 128)))
    assert sel(("se_gate", (32, 32, 320, 320), 4))
    assert sel(("cbam_conv", (32, 64, 160, 160), (128, 4)))
    assert sel(("bias_act", (32, 128, 80, 80), "sum"))  # producer of the SE L23 statistics
    assert sel(plain)  # now the plain variant it is billed against
    assert sel(("conv1x1_thin", (32, 96, 160, 160), (64, "summax")))
    assert sel(("conv1x1_thin", (32, 96, 160, 160), (64, False, False)))
    for key in (("conv3x3", (32, 64, 160, 160), 64), ("conv3x3s2", (32, 64, 160, 160), (128, False, False)),
                ("conv1x1x2", (32, 192, 80, 80), (128, True)), ("bias_act", (32, 64, 80, 80), None)):
        assert not sel(key), key


def test_mafn_path_is_survey_8d_definition():
    """perf.mafn_path: the MAFN instances + decode + NMS scan of SURVEY 8(d), whatever the executor fuses. Synthetic
    region of the n640 paper model (bs 32, one launch each): its HBM floor is 8(d)'s 2.812 GB at 8 TB/s = 0.352 ms;
    the gate-fused SE L1 / CBAM L4 are billed at their 8(d) bytes with the consumer conv's t_min taken off their
    measured time and its FLOPs excluded; the Detect head is billed as the decode."""
    B, nc = 32, 10
    calls = [(("se_conv", (B, 32, 320, 320), (64, 4)), 0.25), (("cbam_conv", (B, 64, 160, 160), (128, 4)), 0.2),
             (("swin", (B, 256, 40, 40), (4, 7, 512)), 0.36), (("a2", (B, 512, 20, 20), (8, 8)), 0.12),
             (("cbam", (B, 256, 40, 40), 16), 0.05), (("se", (B, 128, 80, 80), 8), 0.04),
             (("swin", (B, 64, 160, 160), (2, 7, 128)), 0.45), (("ca", (B, 128, 80, 80), 8), 0.05),
             (("head", (B, 34000), (nc, 64, 64)), 0.15), (("nms", (B, nc, 34000), None), 0.035)]
    ops, _, path = perf.summarize(calls, 1)
    mp = path["mafn"]
    assert abs(mp["t_hbm_floor_ms"] - 0.352) < 2e-3, mp
    assert len(mp["instances"]) == 10
    se8 = perf.t_min_ms(("se", (B, 32, 320, 320), 4), method=True)
    _, t_conv = perf._split_fused(("se_conv", (B, 32, 320, 320), (64, 4)))
    assert 0 < t_conv < 0.25 and se8 < 0.25 - t_conv
    assert abs(mp["t_meas_ms"] - (sum(ms for _, ms in calls) - t_conv
                                  - perf._split_fused(("cbam_conv", (B, 64, 160, 160), (128, 4)))[1])) < 1e-3
    assert mp["frac_vs_hbm_floor"] == round(mp["t_hbm_floor_ms"] / mp["t_meas_ms"], 4)
