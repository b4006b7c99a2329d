"""MI355X-native drop-in for the `latice` VAE hot path (poyentung/ebsd-vae).

Modules this package replaces (same names, classes and call contracts as the reference):
`latice.model`, `latice.lightning_module`, `latice.data_module`, `latice.index.dp_indexer`,
`latice.index.faiss_db`.  Their compute runs in libebsdvae.so (HIP, gfx950) through
`latice._native`.

Modules it does not replace -- `latice.utils` (plotting, IPF colour keys), the Chroma vector
database `latice.index.chroma_db`, the legacy `latice.index.latent_embedding` -- are taken
from a reference checkout when `LATICE_REFERENCE_ROOT` names one (the directory holding the
reference's `latice/` package): its package directories are appended to `__path__`, so this
package's modules win and the reference fills in the rest.  Put `ebsd-vae_amd/` first on
sys.path and point LATICE_REFERENCE_ROOT at the reference root.
"""
import os as _os

__version__ = "0.2.0"

# The training step runs its weight gradients on a second HIP stream; with a data-parallel RCCL
# group initialised, HIP's default of 4 hardware queues per process makes that stream share a
# queue with the main one (the step loses its overlap: 8.55 -> 9.30 ms at B = 256, DESIGN.md
# section 6).  HIP reads the variable when its runtime initialises, so this takes effect when
# latice is imported before the first GPU call; a value the user set is kept.
def _hw_queue_default():
    import sys
    torch = sys.modules.get("torch")
    late = torch is not None and torch.cuda.is_initialized()
    if late and _os.environ.get("GPU_MAX_HW_QUEUES") is None:
        import warnings
        warnings.warn("latice: HIP was initialised before `import latice`, so its default of 4 "
                      "hardware queues per process is in effect; with an RCCL process group the "
                      "weight-gradient stream then shares a queue with the main stream (~0.7 ms "
                      "per step at B = 256). Import latice first, or export GPU_MAX_HW_QUEUES=8.",
                      RuntimeWarning, stacklevel=3)
    _os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")


_hw_queue_default()


def _extend_path(pkg_path, *sub):
    root = _os.environ.get("LATICE_REFERENCE_ROOT")
    if not root:
        return
    d = _os.path.join(root, "latice", *sub)
    if _os.path.isdir(d) and _os.path.realpath(d) not in map(_os.path.realpath, pkg_path):
        pkg_path.append(d)


_extend_path(__path__)
