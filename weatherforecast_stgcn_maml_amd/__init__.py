"""MI355X-native STGCN-LSTM MAML hot path (drop-in for Yalt8826/WeatherForecast_STGCN_MAML's
``model.py`` / ``hybrid_model.py`` / ``train_hybrid_maml_v5.py`` inner/outer loop)."""
from .config import ModelDims, MamlConfig, CONFIG1, CONFIG2  # noqa: F401

__version__ = "0.1.0"
