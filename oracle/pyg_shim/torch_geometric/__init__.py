"""Minimal pure-torch stand-in for torch_geometric==2.0.4 (TEST INFRASTRUCTURE ONLY).

The reference (`/root/reference/src/pathway_explanations`) imports torch_geometric at module
load (data.py:7, model.py:3-4, tests/test_utils.py:7).  The real package (pinned to 2.0.4 by
/root/reference/Dockerfile:13-17 together with torch-scatter 2.0.9 / torch-sparse 0.6.12) is not
installable here.  This shim restates the published PyG 2.0.4 semantics of the handful of
symbols the reference path touches so that `tests/golden/make_golden.py` can import and run the
reference in this container and record golden vectors.

It is never imported by the product package, by `bench.py`'s timed region, or on the GPU box.
"""
from . import nn, utils  # noqa: F401

__version__ = "2.0.4-shim"
