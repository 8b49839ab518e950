"""GPU: weights ingested from a reference-layout checkpoint flow through the HIP path.

The paper model with a trained-like head is written in the reference trainer's layout (save_checkpoint, layout
pinned by tests/test_checkpoint.py against a reference-written file), reloaded with attempt_load_one_weight on the
GPU and on the CPU oracle, and compared: forward within the north-star 1e-3, and NMS (non-empty at conf 0.25 with
these weights) bit-exact against the oracle's NMS on the same predictions."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ckpt_path(tmp_path_factory):
    """Seed-0 paper model whose class-branch output biases are shifted per class (like a trained head: scores
    well above conf 0.25 on many anchors), saved in the reference layout. The rest stays at the well-conditioned
    random init, so CPU and GPU forwards agree to fp32 rounding (fully random weights make the 40-layer forward
    chaotic: 1e-7 differences grow past any fixed tolerance)."""
    import re
    from yolosod_amd.nn.checkpoint import save_checkpoint
    from yolosod_amd.nn.tasks import DetectionModel
    torch.manual_seed(0)
    m = DetectionModel("yolov12-sod-fusion-v5-simple.yaml")
    shift = torch.linspace(6.0, 12.0, m.yaml["nc"])
    with torch.no_grad():
        for k, v in m.state_dict().items():
            if re.fullmatch(r"model\.39\.cv3\.\d\.2\.bias", k):
                v.add_(shift)
    return save_checkpoint(m, tmp_path_factory.mktemp("ck") / "trained_like.pt")


def test_checkpoint_weights_gpu_vs_oracle(ckpt_path, cuda):
    from oracle.model_ref import REGISTRY
    from oracle.nms import non_max_suppression_ref
    from yolosod_amd.utils import ops
    from yolosod_amd.nn.checkpoint import attempt_load_one_weight
    gm, _ = attempt_load_one_weight(ckpt_path, device=cuda)
    cm, _ = attempt_load_one_weight(ckpt_path, device="cpu", registry=REGISTRY)
    g = torch.Generator().manual_seed(5)
    x = torch.rand(2, 3, 640, 640, generator=g)
    with torch.inference_mode():
        y = gm(x.to(cuda))[0]
        ref = cm(x)[0]
    err = (y.cpu() - ref).abs()
    assert float(err.max()) <= 1e-3, float(err.max())
    # NMS on the GPU predictions: HIP kernels vs the oracle on the same tensor
    with torch.inference_mode():
        out, counts, index = ops.non_max_suppression_padded(y.clone(), 0.25, 0.7, max_det=300)
    rows, anchors = non_max_suppression_ref(y.cpu().numpy().copy(), 0.25, 0.7, max_det=300)
    for i in range(2):
        n = int(counts[i])
        assert n == len(rows[i]) and n > 0, (n, len(rows[i]))
        assert np.array_equal(index[i, :n].cpu().numpy(), anchors[i])
        assert np.array_equal(out[i, :n].cpu().numpy(), rows[i])
