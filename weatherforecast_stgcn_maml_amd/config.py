"""Model / MAML configuration mirroring the reference's module-level constants.

Reference: ``train_hybrid_maml_v5.py:20-39`` (model 5.0 constants) and the
checkpoint ``config`` / ``hybrid_config`` dicts (``train_hybrid_maml_v5.py:321-332``).
"""
from __future__ import annotations

from dataclasses import dataclass, asdict, field

# train_hybrid_maml_v5.py:21-38
SEED = 42
NUM_EPOCHS = 40
BATCH_SIZE = 4
INNER_EPOCHS_PER_TASK = 6
INNER_LR = 0.01
OUTER_LR = 0.001
GRAD_ACCUMULATION_STEPS = 2
WINDOW_SIZE = 24
FORECAST_HORIZON = 8
HIDDEN_CHANNELS = 256
LSTM_HIDDEN_SIZE = 128
LSTM_NUM_LAYERS = 4
INPUT_CHANNELS = 12 + 4 + 8
OUTPUT_CHANNELS = 12
INNER_BATCH_CAP = 15          # train_hybrid_maml_v5.py:126 (``if batch_idx >= 15: break``)
MAX_GRAD_NORM = 1.0           # train_hybrid_maml_v5.py:137,176
OUTER_WEIGHT_DECAY = 1e-4     # train_hybrid_maml_v5.py:248

# train_hybrid_maml_v5.py:42-58 (README MODEL_REGIONS)
MODEL_REGIONS = [
    (18, 23, 75, 80),
    (8, 13, 98, 103),
    (53, 58, 35, 40),
    (12.5, 17.5, 102.5, 107.5),
    (22.5, 27.5, 19.5, 24.5),
    (43.5, 48.5, 7.5, 12.5),
    (35.5, 40.5, -5.5, -0.5),
    (32.5, 37.5, 137.5, 142.5),
    (-23.5, -18.5, 132.5, 137.5),
    (-20, -15, -70, -65),
    (44.5, 49.5, 125.5, 130.5),
    (29.5, 34.5, -101.5, -96.5),
    (-9.5, -4.5, -67.5, -62.5),
    (67.5, 72.5, -32.5, -27.5),
    (51.5, 56.5, -112.5, -107.5),
]


@dataclass(frozen=True)
class ModelDims:
    """Shapes of the hybrid STGCN-LSTM (hybrid_model.py:16-58, model.py:8-28)."""

    num_nodes: int = 441
    window_size: int = WINDOW_SIZE
    input_channels: int = INPUT_CHANNELS
    hidden_channels: int = HIDDEN_CHANNELS
    lstm_hidden_size: int = LSTM_HIDDEN_SIZE
    lstm_num_layers: int = LSTM_NUM_LAYERS
    forecast_horizon: int = FORECAST_HORIZON
    output_channels: int = OUTPUT_CHANNELS

    @property
    def head_out(self) -> int:
        return self.forecast_horizon * self.output_channels

    def as_dict(self):
        return asdict(self)


# BASELINE.json configs
CONFIG1 = ModelDims(num_nodes=25, hidden_channels=32, lstm_hidden_size=32, lstm_num_layers=4)
CONFIG2 = ModelDims(num_nodes=441)
# config 5 (stress): N=1024, Hc=512, LSTM kept at 4x128 (interpretation stated in bench output)
CONFIG5 = ModelDims(num_nodes=1024, hidden_channels=512)


@dataclass
class MamlConfig:
    """One meta-step: every task runs ``inner_steps`` SGD steps of ``batch`` samples,
    then one query batch of ``batch`` samples.

    ``order``: 0 = reference semantics (outer update is a no-op, F1),
    1 = first-order MAML, 2 = second-order MAML.
    """

    inner_steps: int = 5
    batch: int = 32
    inner_lr: float = INNER_LR
    max_norm: float = MAX_GRAD_NORM
    order: int = 1
    outer_lr: float = OUTER_LR
    outer_betas: tuple = (0.9, 0.999)
    outer_eps: float = 1e-8
    outer_weight_decay: float = OUTER_WEIGHT_DECAY
    outer_max_norm: float = MAX_GRAD_NORM
    # train_hybrid_maml_v5.py:167: query_loss / GRAD_ACCUMULATION_STEPS
    query_loss_scale: float = 1.0 / GRAD_ACCUMULATION_STEPS
    support_samples: int = 0   # 0 -> inner_steps*batch distinct support samples
    extra: dict = field(default_factory=dict)
