"""Camera helpers (reference: render_video.py:9-19 pose_spherical)."""
import numpy as np
import torch


def pose_spherical(theta: float, phi: float, radius: float) -> torch.Tensor:
    """Camera-to-world [4,4] fp32 looking at the origin from (theta, phi, radius)."""
    def m(rows):
        return torch.tensor(rows, dtype=torch.float32)

    c, s = np.cos(phi / 180.0 * np.pi), np.sin(phi / 180.0 * np.pi)
    rot_phi = m([[1, 0, 0, 0], [0, c, -s, 0], [0, s, c, 0], [0, 0, 0, 1]])
    c, s = np.cos(theta / 180.0 * np.pi), np.sin(theta / 180.0 * np.pi)
    rot_theta = m([[c, 0, -s, 0], [0, 1, 0, 0], [s, 0, c, 0], [0, 0, 0, 1]])
    trans = m([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, radius], [0, 0, 0, 1]])
    flip = m([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]])
    return flip @ (rot_theta @ (rot_phi @ trans))


LEGO_CAMERA_ANGLE_X = 0.6911112070083618


def focal_for(W: int, camera_angle_x: float = LEGO_CAMERA_ANGLE_X) -> float:
    return float(0.5 * W / np.tan(0.5 * camera_angle_x))
