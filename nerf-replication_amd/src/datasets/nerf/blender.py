"""Drop-in ``train/test_dataset_module`` (reference: src/datasets/nerf/blender.py:11-165).

Loads ``transforms_{split}.json`` + RGBA PNGs (PIL), composites onto white
(blender.py:93-95), and keeps the images and camera poses on the GPU.  Instead of the
reference's host table of every ray (1.54 GB for 100 lego views, blender.py:105-108),
rays are generated on demand by the ``nerf_raygen`` kernel from pixel ids: a train item is
a uniform random batch over all pixels of all images (Philox per rank / step), a test
item is one whole image.  Pixel id = img*H*W + j*W + i, the reference's flattening order.

Deliberate difference: the reference draws ``cfg.train.batch_size`` (= 1) rays per step
(blender.py:53,126) while its config's ``N_rays`` is unused; here a train batch has
``cfg.task_arg.train_rays`` rays (default 4096, BASELINE config 3).
"""
import json
import os

import numpy as np
import torch

from nerf_amd import ops
from src.config import cfg


def load_png_rgb(path, W=None, H=None):
    from PIL import Image
    img = Image.open(path)
    if W is not None and (img.width, img.height) != (W, H):
        img = img.resize((W, H), Image.BOX)  # area interpolation (cv2.INTER_AREA)
    a = np.asarray(img).astype(np.float32) / 255.0
    if a.shape[-1] == 4:  # RGBA -> RGB on white (blender.py:93-95)
        a = a[..., :3] * a[..., -1:] + (1.0 - a[..., -1:])
    return a[..., :3]


class Dataset:
    def get_rays(self, H, W, focal, c2w):
        """(rays_o, rays_d) each [H,W,3] for one camera (blender.py:13-32), on c2w's device."""
        dev = c2w.device if c2w.is_cuda else torch.device("cuda")
        pix = torch.arange(H * W, device=dev)
        rays, _, _ = ops.raygen(c2w.to(dev, torch.float32).reshape(1, 4, 4), H, W, focal, pix=pix)
        return rays[:, :3].reshape(H, W, 3), rays[:, 3:].reshape(H, W, 3)

    def __init__(self, **kwargs):
        self.data_root = kwargs.get("data_root")
        self.split = kwargs.get("split", "train")
        self.input_ratio = kwargs.get("input_ratio", 1.0)
        self.cams = kwargs.get("cams", None)
        self.H_orig, self.W_orig = kwargs.get("H"), kwargs.get("W")
        self.device = kwargs.get("device") or torch.device("cuda", torch.cuda.current_device())
        path = os.path.join(self.data_root, cfg.scene, f"transforms_{self.split}.json")
        with open(path, "r") as f:
            meta = json.load(f)
        frames = meta["frames"]
        if self.cams is not None:
            start, stop, step = self.cams
            frames = frames[start:(len(frames) if stop == -1 else stop):step]
        self.H = int(self.H_orig * self.input_ratio)
        self.W = int(self.W_orig * self.input_ratio)
        cam_x = float(meta["camera_angle_x"])
        self.focal = 0.5 * self.W_orig / np.tan(0.5 * cam_x) * self.input_ratio
        imgs, poses = [], []
        for fr in frames:
            p = os.path.join(self.data_root, cfg.scene, fr["file_path"] + ".png")
            imgs.append(load_png_rgb(p, self.W, self.H))
            poses.append(np.asarray(fr["transform_matrix"], dtype=np.float32))
        self.images = torch.from_numpy(np.stack(imgs)).to(self.device)   # [N,H,W,3]
        self.poses = torch.from_numpy(np.stack(poses)).to(self.device)   # [N,4,4]
        self._setup()

    @classmethod
    def from_arrays(cls, images, poses, focal, split="train"):
        """A scene given in memory (synthetic benchmarks, tests)."""
        self = cls.__new__(cls)
        self.split = split
        self.images = images
        self.poses = poses
        self.H, self.W = int(images.shape[1]), int(images.shape[2])
        self.focal = float(focal)
        self.device = images.device
        self._setup()
        return self

    def _setup(self):
        self.n_img = int(self.images.shape[0])
        self.batch_rays = int(cfg.task_arg.get("train_rays", 4096))
        rank = int(os.environ.get("RANK", "0"))
        self.seed = (torch.initial_seed() * 6364136223846793005 + 1442695040888963407 * (rank + 1)) & ((1 << 63) - 1)
        self.draws = 0

    def sample_batch(self, n_rays=None):
        """Uniform random rays over all pixels of all images (blender.py:124-131)."""
        n = n_rays or self.batch_rays
        self.draws += 1
        rays, rgbs, _ = ops.raygen(self.poses, self.H, self.W, self.focal, n_rays=n, seed=self.seed,
                                   offset=self.draws, images=self.images)
        return rays, rgbs

    def image_rays(self, index):
        pix = torch.arange(self.H * self.W, device=self.device) + index * self.H * self.W
        rays, rgbs, _ = ops.raygen(self.poses, self.H, self.W, self.focal, pix=pix, images=self.images)
        return rays, rgbs

    def __getitem__(self, index):
        if self.split == "train":
            rays, rgbs = self.sample_batch()
            ret = {"rays": rays[None], "rgbs": rgbs[None]}
        else:
            rays, rgbs = self.image_rays(index)
            ret = {"rays": rays[None], "rgbs": rgbs[None], "H": torch.tensor([self.H]),
                   "W": torch.tensor([self.W]), "focal": torch.tensor([self.focal])}
        ret["near"] = ops.device_scalar(float(cfg.task_arg.near), self.device)
        ret["far"] = ops.device_scalar(float(cfg.task_arg.far), self.device)
        ret["i"] = torch.tensor([index])
        return ret

    def __len__(self):
        return 1000000 if self.split == "train" else self.n_img
