from dataclasses import dataclass
from typing import List, Optional


@dataclass
class ModelConfig:
    """
    Architecture config for a Two-Tower model
    (reference: pkg/schema/model_config.py:5-25).

    Parameters
    ----------
    joint_embedding_size: int
        Joint embedding size which gets dot product.
    ks: List[int]
        The Recall@k metrics we want to evaluate.
    query_tower_units: Optional[List[int]]
        Hidden units for the query tower.
    candidate_tower_units: Optional[List[int]]
        Hidden units for the candidate tower.
    """

    joint_embedding_size: int
    ks: List[int]
    query_tower_units: Optional[List[int]] = None
    candidate_tower_units: Optional[List[int]] = None
