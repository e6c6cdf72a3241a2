"""Message-passing network (``src/Models/MessagePassingNetwork``), HIP inference path."""
from .model import NodeClassificationMPNSimple, get_mpn_model  # noqa: F401
