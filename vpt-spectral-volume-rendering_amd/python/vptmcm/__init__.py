"""Python harness binding of the MI355X spectral MCM march (libvptmcm.so).

The product host is JavaScript (js/ over napi/); this package is the ctypes
binding that bench.py and the tests use, plus synthetic input generators and
the torch-free multi-process rendezvous used to bootstrap RCCL.
"""
from ._lib import (GROUP_PEER, GROUP_RCCL, MAX_DEVICES, ECOMM, EHIP, EINVAL, ENOMEM, ESTATE, EXPORTS, LAYOUT_BRICK8, LAYOUT_COLUMN4, LAYOUT_CORNER8, LAYOUT_LINEAR, PHOTON_BYTES, PHOTON_RGB_BYTES,
                   RENDERER_RGB, RENDERER_SPECTRAL, Renderer, VptError, lib_path, load, unique_id)

__all__ = ["GROUP_PEER", "GROUP_RCCL", "MAX_DEVICES", "ECOMM", "EHIP", "EINVAL", "ENOMEM", "ESTATE", "EXPORTS", "LAYOUT_BRICK8", "LAYOUT_COLUMN4", "LAYOUT_CORNER8", "LAYOUT_LINEAR", "PHOTON_BYTES", "PHOTON_RGB_BYTES",
           "RENDERER_RGB", "RENDERER_SPECTRAL", "Renderer", "VptError", "lib_path", "load",
           "unique_id"]
