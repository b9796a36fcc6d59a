"""Drop-in ``evaluator_module`` (reference: src/evaluators/nerf.py:16-92).

PSNR on the float images (nerf.py:23-26) and SSIM on uint8 images with
data_range = pred.max() - pred.min() (nerf.py:28-45).  scikit-image is not installed in
this image, so ``structural_similarity`` is restated from its documented defaults
(7x7 uniform window via scipy.ndimage.uniform_filter in 'reflect' mode, K1 = 0.01,
K2 = 0.03, sample covariance N/(N-1), border of 3 px cropped before the mean, mean over
channels).  Parity of this restatement with scikit-image is unpinned here (no skimage
to compare against).  PNG dumps use PIL instead of cv2.

When the rendered image is on the GPU (run.py --type evaluate, Trainer.val) the metrics
run there (``nerf_image_metrics``, csrc/metrics.hip: exact integer window sums, fp64 SSIM
formula), and the PNG dump (save_result, the reference's default) is written from the uint8
images converted on the device: one 1.9 MB copy per 800x800 view instead of the float image
and a host SSIM.  The numpy functions below are the same definitions on the host (used for
host images and as the GPU kernel's test reference).
"""
import json
import os

import numpy as np
import torch
from scipy.ndimage import uniform_filter

from src.config import cfg


def psnr_metric(pred, gt):
    mse = np.mean((pred - gt) ** 2)
    return -10 * np.log(mse) / np.log(10)


def ssim_channel(x, y, data_range, win=7, K1=0.01, K2=0.03):
    x = x.astype(np.float64)
    y = y.astype(np.float64)
    ux, uy = uniform_filter(x, size=win), uniform_filter(y, size=win)
    uxx, uyy, uxy = uniform_filter(x * x, size=win), uniform_filter(y * y, size=win), uniform_filter(x * y, size=win)
    n = win ** 2
    cov = n / (n - 1.0)
    vx, vy, vxy = cov * (uxx - ux * ux), cov * (uyy - uy * uy), cov * (uxy - ux * uy)
    C1, C2 = (K1 * data_range) ** 2, (K2 * data_range) ** 2
    S = ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux ** 2 + uy ** 2 + C1) * (vx + vy + C2))
    pad = (win - 1) // 2
    return S[pad:-pad, pad:-pad].mean()


def ssim_metric_uint8(pred_u8, gt_u8):
    data_range = float(pred_u8.max()) - float(pred_u8.min())
    return float(np.mean([ssim_channel(pred_u8[..., c], gt_u8[..., c], data_range) for c in range(pred_u8.shape[-1])]))


class Evaluator:
    def __init__(self):
        self.mse, self.psnr, self.ssim = [], [], []
        self.save_images = cfg.get("save_result", True)

    def psnr_metric(self, img_pred, img_gt):
        return psnr_metric(img_pred, img_gt)

    @staticmethod
    def png_pixels(img_pred, img_gt_u8):
        """The pixel values the reference's cv2.imwrite calls store (nerf.py:31-38): the float
        prediction x 255 converted by OpenCV's saturate_cast (round half to even, clamp to
        [0, 255]); the ground truth is already uint8 there, and its ``* 255`` stays uint8 and
        wraps modulo 256 (NumPy keeps the array's dtype for a Python int operand), so the
        reference's gt PNG holds (255 g) mod 256 -- reproduced as written."""
        pred = np.clip(np.rint(img_pred.astype(np.float32) * np.float32(255)), 0, 255).astype(np.uint8)
        return pred, (img_gt_u8 * 255).astype(np.uint8)

    def save_pngs(self, pred_u8, gt_u8, id):
        """view{id}_pred.png / _gt.png under result_dir/images (nerf.py:29-38 of the reference);
        pixel values as png_pixels gives them."""
        from PIL import Image
        d = os.path.join(cfg.result_dir, "images")
        os.makedirs(d, exist_ok=True)
        Image.fromarray(pred_u8).save(f"{d}/view{id:03d}_pred.png")
        Image.fromarray(gt_u8).save(f"{d}/view{id:03d}_gt.png")

    def ssim_metric(self, img_pred, img_gt, batch, id, num_imgs):
        if self.save_images:
            self.save_pngs(*self.png_pixels(img_pred, img_gt), id)
        return ssim_metric_uint8((img_pred * 255).astype(np.uint8), img_gt)

    def evaluate(self, output, batch):
        i = int(batch["i"].reshape(-1)[0])
        H, W = int(batch["H"].reshape(-1)[0]), int(batch["W"].reshape(-1)[0])
        pred_t = output["rgb_map_f"].detach().float()
        gt_t = batch["rgbs"].detach().float()
        if pred_t.is_cuda and gt_t.is_cuda:
            from nerf_amd import ops
            pred_t, gt_t = pred_t.reshape(H, W, 3), gt_t.reshape(H, W, 3)
            psnr, ssim = ops.image_metrics(pred_t, gt_t)
            if self.save_images:  # png_pixels on the device: one uint8 copy per image
                pred_png = torch.round(pred_t * 255).clamp(0, 255).to(torch.uint8)
                gt_png = ((gt_t * 255).to(torch.uint8).to(torch.int32) * 255 % 256).to(torch.uint8)
                self.save_pngs(pred_png.cpu().numpy(), gt_png.cpu().numpy(), i)
            self.psnr.append(psnr)
            self.ssim.append(ssim)
            return {"psnr": psnr, "ssim": ssim}
        pred = pred_t.cpu().numpy()
        gt = gt_t.cpu().numpy().reshape(-1, 3)
        img_pred, img_gt = pred.reshape(H, W, 3), gt.reshape(H, W, 3)
        psnr = self.psnr_metric(img_pred, img_gt)
        ssim = self.ssim_metric(img_pred, (img_gt * 255).astype(np.uint8), batch, i, 100)
        self.psnr.append(psnr)
        self.ssim.append(ssim)
        return {"psnr": psnr, "ssim": ssim}

    def summarize(self):
        mean_psnr, mean_ssim = float(np.mean(self.psnr)), float(np.mean(self.ssim))
        print("Final Evaluation Results:")
        print(f"  Average PSNR: {mean_psnr:.4f}")
        print(f"  Average SSIM: {mean_ssim:.4f}")
        os.makedirs(cfg.result_dir, exist_ok=True)
        path = os.path.join(cfg.result_dir, "summary.json")
        with open(path, "w") as f:
            json.dump({"mean_psnr": mean_psnr, "mean_ssim": mean_ssim}, f, indent=4)
        print(f"\nSummary saved to {path}")
        self.psnr, self.ssim = [], []
        return {"psnr": mean_psnr, "ssim": mean_ssim}
