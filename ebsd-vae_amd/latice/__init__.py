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


def _extend_path(pkg_path, *sub):
    root = _os.environ.get("LATICE_REFERENCE_ROOT")
    if not root:
        return
    d = _os.path.join(root, "latice", *sub)
    if _os.path.isdir(d) and _os.path.realpath(d) not in map(_os.path.realpath, pkg_path):
        pkg_path.append(d)


_extend_path(__path__)
