"""commefficient_amd: communication-efficient federated SGD, MI355X-native."""
import os as _os


def request_graph_replay() -> bool:
    """Opt in to HIP-graph replay (``--graph on|auto``, parallel/graph.py).

    ROCm 7.2's ROCclr pre-builds the AQL packets of a HIP graph at
    instantiation ("graph packet capture"); with it, the SECOND launch of the
    captured ResNet-9 round graph raised a memory-access fault in round 1
    (the first launch was bitwise identical to eager execution).  With the
    capture off (``DEBUG_CLR_GRAPH_PACKET_CAPTURE=0``) graphs launch through
    the regular dispatch path and replay correctly.  The variable is read when
    the HIP runtime initialises, so it is set only here, only when graph replay
    is requested, and only if HIP is not initialised yet -- never on import,
    since it changes the behaviour of every graph in the process.  Returns
    whether graph replay can be used."""
    if _os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") == "0":
        return True
    import torch
    if torch.cuda.is_initialized():
        return False
    _os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] = "0"
    return True
