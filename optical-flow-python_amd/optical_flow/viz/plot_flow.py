"""Flow plotting (host-side; reference: optical_flow/viz/plot_flow.py). matplotlib is optional."""
import numpy as np

from optical_flow.viz.flow_color import flow_to_color


def plot_flow(uv, method='color', max_flow=None, ax=None, title=None, step=None):
    import matplotlib.pyplot as plt  # optional dependency
    if ax is None:
        _, ax = plt.subplots(1, 1)
    if method == 'color':
        ax.imshow(flow_to_color(uv, max_flow))
    else:
        H, W = uv.shape[:2]
        s = step or max(1, min(H, W) // 32)
        y, x = np.mgrid[0:H:s, 0:W:s]
        ax.quiver(x, y, uv[::s, ::s, 0], -uv[::s, ::s, 1])
        ax.invert_yaxis()
    if title:
        ax.set_title(title)
    ax.axis('off')
    return ax
