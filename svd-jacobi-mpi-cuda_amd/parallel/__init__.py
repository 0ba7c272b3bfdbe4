"""Schedules, communicator (torch.distributed: RCCL on GPU, gloo on CPU) and
the distributed block-Jacobi solver."""
from . import pipeline, schedule  # noqa: F401
from .comm import Communicator, SimCommunicator  # noqa: F401,E402
from .distributed import DistributedBlockJacobi  # noqa: F401,E402
