"""MI355X-native drop-in for the `latice` VAE hot path (poyentung/ebsd-vae).

Public modules mirror the reference: `latice.model`, `latice.lightning_module`.
The compute runs in libebsdvae.so (HIP, gfx950) through `latice._native`.
"""
__version__ = "0.1.0"
