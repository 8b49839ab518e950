"""ORACLE - TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's hot path (quitedob/yolo-sod): ``ops_ref`` (MAFN operators + Detect decode,
PyTorch-CPU math), ``nms`` + ``nms_ref.c`` (non_max_suppression around a C restatement of torchvision's CPU NMS),
``model_ref`` (whole model with these operators). Pinned by the golden fixtures in ``tests/golden/`` generated from
the reference itself. Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import it - as the checker, never as the measured or shipped path.
"""
