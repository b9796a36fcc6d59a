"""The drop-in Evaluator on its default path (reference src/evaluators/nerf.py:23-92, called by
run.py --type evaluate and Trainer.val): a rendered image on the device is scored on the GPU
(nerf_image_metrics) even with the PNG dump on (save_result, the reference's default), and the
PNGs come from the uint8 images converted on the device.  Checked against the same Evaluator
fed host arrays (its numpy definitions: PSNR nerf.py:23-26, the skimage-default SSIM restated):
PSNR within 1e-4 dB, SSIM within 1e-9, identical PNG bytes, summary.json written."""
import json
import os

import numpy as np
import pytest
import torch
from PIL import Image

pytestmark = pytest.mark.gpu
os.environ.setdefault("NERF_AMD_NO_ARGV", "1")


def test_evaluator_default_path_on_gpu(cuda, tmp_path):
    from src.config import cfg
    from src.evaluators import nerf as ev_mod
    old = cfg.result_dir
    cfg.result_dir = str(tmp_path / "gpu")
    try:
        H, W = 120, 96
        g = torch.Generator().manual_seed(5)
        gt = torch.rand(1, H * W, 3, generator=g)
        pred = (gt[0] + 0.07 * torch.randn(H * W, 3, generator=g)).clamp(0.0, 1.0)
        batch = {"i": torch.tensor([3]), "H": torch.tensor([H]), "W": torch.tensor([W])}
        e = ev_mod.Evaluator()
        assert e.save_images  # the reference's behaviour: PNGs are written
        calls = []
        from nerf_amd import ops
        real = ops.image_metrics
        ops.image_metrics = lambda *a: calls.append(1) or real(*a)
        try:
            got = e.evaluate({"rgb_map_f": pred.to(cuda)}, dict(batch, rgbs=gt.to(cuda)))
        finally:
            ops.image_metrics = real
        assert calls == [1]  # scored on the GPU
        gdir = tmp_path / "gpu" / "images"
        cfg.result_dir = str(tmp_path / "host")
        host = ev_mod.Evaluator().evaluate({"rgb_map_f": pred}, dict(batch, rgbs=gt))
        hdir = tmp_path / "host" / "images"
        assert abs(got["psnr"] - host["psnr"]) < 1e-4, (got, host)
        assert abs(got["ssim"] - host["ssim"]) < 1e-9, (got, host)
        for name in ("view003_pred.png", "view003_gt.png"):
            np.testing.assert_array_equal(np.asarray(Image.open(gdir / name)), np.asarray(Image.open(hdir / name)))
        # the reference's cv2.imwrite values: saturate_cast (round half to even) of pred x 255,
        # and its uint8 gt x 255 wrapped modulo 256
        p32 = pred.reshape(H, W, 3).numpy()
        np.testing.assert_array_equal(np.asarray(Image.open(gdir / "view003_pred.png")),
                                      np.clip(np.rint(p32 * np.float32(255)), 0, 255).astype(np.uint8))
        g8 = (gt.reshape(H, W, 3).numpy() * 255).astype(np.uint8)
        np.testing.assert_array_equal(np.asarray(Image.open(gdir / "view003_gt.png")),
                                      ((g8.astype(np.int64) * 255) % 256).astype(np.uint8))
        cfg.result_dir = str(tmp_path / "gpu")
        s = e.summarize()
        with open(tmp_path / "gpu" / "summary.json") as f:
            saved = json.load(f)
        assert saved["mean_psnr"] == pytest.approx(s["psnr"]) and saved["mean_ssim"] == pytest.approx(s["ssim"])
    finally:
        cfg.result_dir = old
