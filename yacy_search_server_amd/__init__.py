"""yrwi -- MI355X-native YaCy RWI query hot path (join -> normalise -> cardinal -> top-k).

The compute path is libyrwi.so (hand-written HIP for gfx950, C ABI in
include/yrwi.h); `rwi` mirrors YaCy's Java API over it and `synth` generates
the synthetic RWI corpora of BASELINE.md."""

from .rwi import Hit, Query, QueryFilter, RankingProfile, RWIIndex, SearchEvent, unique_id  # noqa: F401
