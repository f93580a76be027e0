"""Data-parallel training: engine, communicators, launcher, trainer."""
from .comm import Communicator, NullComm, TorchDistComm, LoopbackComm  # noqa: F401
from .engine import MlpEngine, FlatLayout  # noqa: F401
from .trainer import DataParallelTrainer, parallel_train, TrainStats  # noqa: F401
from .tensor_parallel import TensorParallelTrainer  # noqa: F401
