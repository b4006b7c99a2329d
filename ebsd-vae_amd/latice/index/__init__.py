"""EBSD pattern indexer on the MI355X path (latice/index in the reference).

`dp_indexer.DiffractionPatternIndexer` keeps the reference's API and call contracts;
`faiss_db.FaissLatentVectorDatabase` keeps the FAISS-backed API (latice/index/faiss_db.py)
with the dictionary resident in HBM: exact cosine top-k and the orientation consensus run as
HIP kernels (csrc/search.hip, csrc/orient.hip).  Other reference modules of this package
(chroma_db, latent_embedding) resolve from LATICE_REFERENCE_ROOT (see latice/__init__.py).
"""
from latice import _extend_path

_extend_path(__path__, "index")
