"""Cluster bring-up helpers (reference ``deploy/determined_deploy/local/cluster_utils.py``)."""
from determined_1_amd.deploy.local import LocalCluster, native_binary

__all__ = ["LocalCluster", "native_binary"]
