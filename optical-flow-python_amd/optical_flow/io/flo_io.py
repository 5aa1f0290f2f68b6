"""Middlebury .flo I/O (host-side; reference: optical_flow/io/flo_io.py:15-113).

Layout: float32 tag 202021.25, int32 width, int32 height, then H*W*2 float32
(u, v interleaved, row-major)."""
import os

import numpy as np

TAG_FLOAT = 202021.25


def read_flo(filename):
    with open(filename, 'rb') as f:
        head = f.read(12)
        if len(head) < 12:
            raise ValueError(f"Invalid .flo file: {filename} is too short")
        tag = np.frombuffer(head[:4], np.float32)[0]
        if tag != TAG_FLOAT:
            raise ValueError(f'Invalid .flo file tag: {tag} (expected {TAG_FLOAT})')
        w, h = np.frombuffer(head[4:], np.int32)
        data = np.fromfile(f, np.float32)
    return data.reshape((int(h), int(w), 2))


def write_flo(flow, filename):
    flow = np.asarray(flow, dtype=np.float32)
    if flow.ndim != 3 or flow.shape[2] != 2:
        raise ValueError(f"Flow must be (H, W, 2) array, got shape {flow.shape}")
    h, w = flow.shape[:2]
    with open(filename, 'wb') as f:
        f.write(np.float32(TAG_FLOAT).tobytes())
        f.write(np.array([w, h], dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(flow).tobytes())


def read_flow_file(seq_name, i_seq, data_dir=None):
    """frame{i}.png, frame{i+1}.png and flow{i}.flo of a Middlebury sequence
    laid out as data_dir/other-data/<seq>/ and data_dir/other-gt-flow/<seq>/."""
    from PIL import Image
    if data_dir is None:
        data_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(__file__))), 'data')
    img_dir = os.path.join(data_dir, 'other-data', seq_name)
    im1 = np.array(Image.open(os.path.join(img_dir, f'frame{i_seq:02d}.png'))).astype(np.float64)
    im2 = np.array(Image.open(os.path.join(img_dir, f'frame{i_seq + 1:02d}.png'))).astype(np.float64)
    gt_path = os.path.join(data_dir, 'other-gt-flow', seq_name, f'flow{i_seq:02d}.flo')
    if os.path.exists(gt_path):
        gt = read_flo(gt_path)
        return im1, im2, gt[:, :, 0], gt[:, :, 1]
    return im1, im2, None, None
