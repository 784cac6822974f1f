from .cluster_spec import ClusterSpec, RankLayout, parse_host_list, split_address
from .server import Server, current
from .launcher import maybe_spawn_towers, launch_local_cluster, under_torchrun, is_tower_child

__all__ = ["ClusterSpec", "RankLayout", "parse_host_list", "split_address", "Server", "current",
           "maybe_spawn_towers", "launch_local_cluster", "under_torchrun", "is_tower_child"]
