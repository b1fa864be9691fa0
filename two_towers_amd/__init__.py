"""two_towers_amd — MI355X-native two-tower contrastive training step.

Drop-in for the hot path of mateomarin/two_towers (train_enhanced.py:54-69): the
EnhancedTwoTowerModel / InfoNCELoss / MarginRankingLoss / get_hard_negatives surface
of enhanced_two_tower.py (and the margin family of margin_two_tower.py in .margin, the
/search service in .serving), computed by hand-written HIP kernels for gfx950
(libtt_hip.so, C ABI in include/tt_hip.h). There is no CPU fallback.
"""
from .data import (EnhancedDataset, EnhancedIdDataset, MSMarcoDataset, Vocab, encode_batch, encode_ids,
                   load_ms_marco_train, load_word2vec, pairs_from_msmarco)
from .margin import MarginIdDataset, SimpleDataset, TwoTowerModel, margin_ids
from .losses import HardNegativeMarginLoss, InfoNCELoss, MarginRankingLoss, get_hard_negatives, mine_hard_negatives
from .model import EnhancedTwoTower, EnhancedTwoTowerModel
from .optim import Adam
from ._lib import GruTimeoutError
from .towers import check_gru_status

__all__ = [
    "EnhancedTwoTowerModel", "EnhancedTwoTower", "InfoNCELoss", "MarginRankingLoss", "HardNegativeMarginLoss",
    "get_hard_negatives", "mine_hard_negatives", "EnhancedDataset", "EnhancedIdDataset", "MSMarcoDataset",
    "Vocab", "encode_ids", "encode_batch", "load_word2vec", "load_ms_marco_train", "pairs_from_msmarco", "Adam",
    "TwoTowerModel", "SimpleDataset", "MarginIdDataset", "margin_ids", "check_gru_status", "GruTimeoutError",
]
__version__ = "0.1.0"
