"""EBSD pattern indexer pieces on the MI355X path (latice/index in the reference).

`faiss_db.FaissLatentVectorDatabase` keeps the reference's FAISS-backed API
(latice/index/faiss_db.py) with the dictionary resident in HBM: exact cosine top-k and the
orientation consensus run as HIP kernels (csrc/search.hip, csrc/orient.hip).
"""
