"""commefficient_amd: communication-efficient federated SGD, MI355X-native."""
import os as _os

# ROCm 7.2's ROCclr builds the AQL packets of a HIP graph once at
# instantiation ("graph packet capture"); with it, the SECOND launch of the
# captured round graph (parallel/graph.py) raises a memory-access fault while
# the first launch is bitwise identical to eager execution.  With the packet
# capture off, graphs launch through the regular dispatch path and replay
# correctly.  Read when the HIP runtime initialises, so set on import.
_os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
