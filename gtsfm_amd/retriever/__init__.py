"""Image-pair retrievers (gtsfm/retriever/): which pairs the two-view front-end matches."""
from gtsfm_amd.retriever.retriever_base import ImageMatchingRegime, RetrieverBase  # noqa: F401
from gtsfm_amd.retriever.sequential_retriever import ExhaustiveRetriever, SequentialRetriever  # noqa: F401
