"""Launch / cluster resolution: torchrun, Open MPI / horovodrun, SLURM, and
the in-process cluster of the parameter-server script.

Reference call sites:
  * SlurmClusterResolver(port_base=12345) + int(os.environ['SLURM_NTASKS'])
    (imagenet-resnet50-multiworkers.py:16,29)
  * hvd.init() / hvd.rank() / hvd.size() / hvd.local_rank() (imagenet-resnet50-hvd.py:16,39-41)
  * create_in_process_cluster(num_workers, num_ps) with portpicker ports
    (imagenet-resnet50-ps.py:31-65)
Every resolver yields the same `ClusterInfo`; rendezvous always uses 127.0.0.1 for
single-node jobs (the container hostname may not resolve).
"""
from __future__ import annotations

import os
import re
import socket
from dataclasses import dataclass, field
from typing import Dict, List, Optional


@dataclass
class ClusterInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    master_addr: str = "127.0.0.1"
    master_port: int = 29500
    source: str = "single"
    hosts: List[str] = field(default_factory=lambda: ["127.0.0.1"])
    task_addresses: List[str] = field(default_factory=list)   # SLURM: host:port per task

    @property
    def is_chief(self) -> bool:
        return self.rank == 0


def expand_hostlist(spec: str) -> List[str]:
    """SLURM hostlist expression -> host names: 'n[01-03,07],gpu5' -> n01 n02 n03 n07 gpu5."""
    out: List[str] = []
    for part in re.findall(r"[^,\[]+(?:\[[^\]]*\])?[^,]*", spec):
        part = part.strip(",")
        if not part:
            continue
        m = re.match(r"^(.*?)\[([^\]]*)\](.*)$", part)
        if not m:
            out.append(part)
            continue
        pre, body, post = m.groups()
        for rng in body.split(","):
            if "-" in rng:
                a, b = rng.split("-")
                w = len(a)
                for i in range(int(a), int(b) + 1):
                    out.append(f"{pre}{str(i).zfill(w)}{post}")
            else:
                out.append(f"{pre}{rng}{post}")
    return out


def expand_tasks_per_node(spec: str) -> List[int]:
    """'2(x3),1' -> [2, 2, 2, 1]"""
    out: List[int] = []
    for tok in spec.split(","):
        m = re.match(r"^(\d+)(?:\(x(\d+)\))?$", tok.strip())
        if not m:
            raise ValueError(f"bad SLURM tasks-per-node spec {spec!r}")
        out += [int(m.group(1))] * int(m.group(2) or 1)
    return out


class SlurmClusterResolver:
    """Mirror of tf.distribute.cluster_resolver.SlurmClusterResolver(port_base=...): every
    task gets host:port_base+local_index; task 0 is the chief / rendezvous master."""

    def __init__(self, port_base: int = 12345, env: Optional[Dict[str, str]] = None,
                 gpus_per_node: Optional[int] = None):
        self.env = dict(os.environ if env is None else env)
        self.port_base = port_base
        self.gpus_per_node = gpus_per_node

    def resolve(self) -> ClusterInfo:
        e = self.env
        rank = int(e["SLURM_PROCID"])
        ntasks = int(e.get("SLURM_STEP_NUM_TASKS", e.get("SLURM_NTASKS", "1")))
        nodes = expand_hostlist(e.get("SLURM_STEP_NODELIST", e.get("SLURM_JOB_NODELIST", "localhost")))
        tpn = expand_tasks_per_node(e.get("SLURM_STEP_TASKS_PER_NODE", e.get("SLURM_TASKS_PER_NODE",
                                                                            str(ntasks))))
        if len(tpn) < len(nodes):
            tpn += [tpn[-1]] * (len(nodes) - len(tpn))
        addrs = []
        for host, n in zip(nodes, tpn):
            for i in range(n):
                addrs.append(f"{host}:{self.port_base + i}")
        addrs = addrs[:ntasks]
        local_rank = int(e.get("SLURM_LOCALID", "0"))
        node_idx = int(e.get("SLURM_NODEID", "0"))
        local_world = tpn[node_idx] if node_idx < len(tpn) else 1
        master = nodes[0]
        if len(nodes) == 1:
            master = "127.0.0.1"
        return ClusterInfo(rank=rank, world_size=ntasks, local_rank=local_rank, local_world_size=local_world,
                           master_addr=master, master_port=self.port_base, source="slurm", hosts=nodes,
                           task_addresses=addrs)


def resolve_cluster(env: Optional[Dict[str, str]] = None, port_base: int = 12345) -> ClusterInfo:
    """torchrun > Open MPI (mpirun/horovodrun) > SLURM > single process."""
    e = dict(os.environ if env is None else env)
    if "RANK" in e and "WORLD_SIZE" in e:
        return ClusterInfo(rank=int(e["RANK"]), world_size=int(e["WORLD_SIZE"]),
                           local_rank=int(e.get("LOCAL_RANK", "0")),
                           local_world_size=int(e.get("LOCAL_WORLD_SIZE", e["WORLD_SIZE"])),
                           master_addr=e.get("MASTER_ADDR", "127.0.0.1"),
                           master_port=int(e.get("MASTER_PORT", "29500")), source="torchrun")
    if "OMPI_COMM_WORLD_RANK" in e:
        return ClusterInfo(rank=int(e["OMPI_COMM_WORLD_RANK"]), world_size=int(e["OMPI_COMM_WORLD_SIZE"]),
                           local_rank=int(e.get("OMPI_COMM_WORLD_LOCAL_RANK", "0")),
                           local_world_size=int(e.get("OMPI_COMM_WORLD_LOCAL_SIZE", "1")),
                           master_addr=e.get("MASTER_ADDR", "127.0.0.1"),
                           master_port=int(e.get("MASTER_PORT", "29500")), source="mpi")
    if "SLURM_PROCID" in e and int(e.get("SLURM_NTASKS", e.get("SLURM_STEP_NUM_TASKS", "1"))) > 1:
        return SlurmClusterResolver(port_base, e).resolve()
    return ClusterInfo()


def export_torch_env(info: ClusterInfo) -> None:
    """Make `torch.distributed.init_process_group('env://')` see the resolved cluster."""
    os.environ["RANK"] = str(info.rank)
    os.environ["WORLD_SIZE"] = str(info.world_size)
    os.environ["LOCAL_RANK"] = str(info.local_rank)
    os.environ["LOCAL_WORLD_SIZE"] = str(info.local_world_size)
    os.environ.setdefault("MASTER_ADDR", info.master_addr)
    os.environ.setdefault("MASTER_PORT", str(info.master_port))


def pick_unused_port() -> int:
    """portpicker.pick_unused_port() equivalent (imagenet-resnet50-ps.py:33-34)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def create_in_process_cluster(num_workers: int, num_ps: int) -> Dict[str, List[str]]:
    """ClusterSpec dict {"worker": [...], "ps": [...]} on localhost with free ports
    (imagenet-resnet50-ps.py:31-41).  The PS strategy starts one role per entry."""
    spec = {"worker": [f"127.0.0.1:{pick_unused_port()}" for _ in range(num_workers)]}
    if num_ps > 0:
        spec["ps"] = [f"127.0.0.1:{pick_unused_port()}" for _ in range(num_ps)]
    return spec
