"""MI355X-native variational optical flow.

Drop-in for jordanshivers/optical-flow-python: same estimate_flow() /
compute_flow() API and method registry; the coarse-to-fine IRLS hot path runs
as hand-written HIP kernels for gfx950 in liboptflow.so (include/optflow.h).
"""
from optical_flow.interface import estimate_flow, estimate_flow_batch, PairStream
from optical_flow.io.flo_io import read_flo, write_flo
from optical_flow.viz.flow_color import flow_to_color
from optical_flow.viz.plot_flow import plot_flow
from optical_flow.evaluation.metrics import flow_angular_error
from optical_flow.methods.config import load_of_method

__all__ = ['estimate_flow', 'estimate_flow_batch', 'PairStream', 'read_flo', 'write_flo', 'flow_to_color', 'plot_flow', 'flow_angular_error',
           'load_of_method']
