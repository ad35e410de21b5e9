"""Synthetic MI355X node fixtures (sysfs + /dev trees).

The reference only has captured trees of older parts (MI210, MI300X CPX,
MI308X) and its discovery cannot even read them because its
paths are hard-coded. This generator writes a complete, self-consistent
8x MI355X (gfx950, gfx_target_version 90500, 288 GiB HBM3E, 256 CUs / 8 XCDs
per GPU) node in any compute partition mode (SPX/DPX/QPX/CPX: 1/2/4/8
partitions per GPU) and memory mode (NPS1/NPS2), with:

* kfd topology: CPU nodes + one GPU node per partition, properties,
  io_links (xGMI inside a hive, PCIe to the CPU), p2p_links (PCIe across hives),
  mem_banks;
* amdgpu PCI functions (``module/amdgpu/drivers/pci:amdgpu/<BDF>`` symlinks
  into ``devices/pci0000:00``) with partition files, numa_node and drm nodes;
* ``devices/platform/amdgpu_xcp_<N>`` for the partitions beyond the first;
* ``class/drm/card<N>/device`` links with vendor/device/product_name and
  driver module version;
* optional SR-IOV (gim + virtfn) or vfio-pci passthrough PCI trees;
* a matching ``dev`` tree (kfd, dri/card*, dri/renderD*, vfio/*).

Everything here is synthetic; exact MI355X sysfs strings should be confirmed
on hardware (the GPU tests compare this layout with the real box).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional, Sequence

from ..models import MI355X

PARTITIONS = {cp: MI355X.partitions_per_gpu(cp) for cp in MI355X.compute_partitions}
MI355X_DEVICE_ID = MI355X.device_ids[0]
MI355X_VF_DEVICE_ID = MI355X.vf_device_ids[0]
MI355X_PRODUCT = MI355X.name
MI355X_VRAM = MI355X.vram_bytes
MI355X_CUS = MI355X.cus
MI355X_XCDS = MI355X.xcds
DEFAULT_BUSES = [0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xE5, 0xF5]


@dataclass
class FixtureSpec:
    num_gpus: int = 8
    compute_partition: str = "spx"
    memory_partition: str = "nps1"
    numa_nodes: int = 2
    cpus_per_numa: int = 64
    cpu_dirs_per_numa: int = 2  # CPUs materialised under devices/system/{node,cpu} (keeps fixtures small)
    hive_size: int = 8                  # GPUs per xGMI hive (8 = one hive)
    gfx_target_version: int = 90500
    device_id: int = MI355X_DEVICE_ID
    product_name: str = MI355X_PRODUCT
    driver_version: str = "6.12.12"
    driver_srcversion: str = "A1B2C3D4E5F60718293A4B5"
    mode: str = "container"             # container | vf | pf
    vfs_per_gpu: int = 1                # SR-IOV VFs per PF (mode="vf")
    partition_support: bool = True      # write available_*_partition files
    per_gpu_compute: Optional[List[str]] = None  # heterogeneous nodes
    generation: int = 1                 # kfd topology generation_id (bump to emulate a reconfiguration)
    # "compact": one amdgpu_xcp_<8g+p> per extra partition, drm minors numbered
    # over active partitions only (the reference test-ID scheme).
    # "kernel": what amdgpu does (amdgpu_xcp_dev_alloc; measured on the MI355X
    # box, profiles/archive/sysfs_access_box.json): every GPU owns a block of 8 drm
    # minors in probe order (its own + 7 amdgpu_xcp_* devices, present even in
    # SPX), xcp index 7*rank + slot - 1; inactive slots have no kfd node.
    xcp_layout: str = "compact"
    probe_order: Optional[List[int]] = None  # kernel layout: GPU indices in driver probe order


@dataclass
class FixtureInfo:
    root: Path
    sysfs: Path
    dev: Path
    device_ids: List[str] = field(default_factory=list)
    bdfs: List[str] = field(default_factory=list)
    unique_ids: List[str] = field(default_factory=list)
    hive_ids: List[int] = field(default_factory=list)
    render_minors: Dict[str, int] = field(default_factory=dict)
    node_ids: Dict[str, int] = field(default_factory=dict)
    gpu_of: Dict[str, int] = field(default_factory=dict)   # device ID -> GPU index


def _w(path: Path, content: str) -> None:
    path.parent.mkdir(parents=True, exist_ok=True)
    path.write_text(content if content.endswith("\n") else content + "\n")


def _link(target: Path, link: Path) -> None:
    link.parent.mkdir(parents=True, exist_ok=True)
    if link.is_symlink() or link.exists():
        link.unlink()
    os.symlink(os.path.relpath(target, link.parent), link)


def _props(kv: Sequence) -> str:
    return "\n".join(f"{k} {v}" for k, v in kv)


def _unique_id(g: int) -> str:
    # stable 64-bit-ish ids, like kfd's (decimal)
    return str((0x9E3779B97F4A7C15 * (g + 1)) % (2 ** 64))


def _hive_id(h: int) -> int:
    return (0xC2B2AE3D27D4EB4F * (h + 7)) % (2 ** 64)


def make_mi355x_node(root: os.PathLike, spec: Optional[FixtureSpec] = None, **kw) -> FixtureInfo:
    spec = spec or FixtureSpec(**kw)
    root = Path(root)
    sysfs = root / "sys"
    dev = root / "dev"
    info = FixtureInfo(root=root, sysfs=sysfs, dev=dev)
    nodes_dir = sysfs / "class/kfd/kfd/topology/nodes"
    pci_root = sysfs / "devices/pci0000:00"
    drv_amdgpu = sysfs / "bus/pci/drivers/amdgpu"
    _w(sysfs / "module/amdgpu/version", spec.driver_version)
    _w(sysfs / "module/amdgpu/srcversion", spec.driver_srcversion)
    (sysfs / "module/amdgpu/drivers").mkdir(parents=True, exist_ok=True)
    drv_amdgpu.mkdir(parents=True, exist_ok=True)
    _link(sysfs / "module/amdgpu", drv_amdgpu / "module")
    _link(drv_amdgpu, sysfs / "module/amdgpu/drivers/pci:amdgpu")
    dev.mkdir(parents=True, exist_ok=True)
    (dev / "dri").mkdir(exist_ok=True)
    _w(dev / "kfd", "")
    if spec.mode == "container":
        _w(sysfs / "class/kfd/kfd/topology/generation_id", str(spec.generation))

    numa = max(1, spec.numa_nodes)
    # host NUMA/CPU sysfs (a few CPUs per node, each with cache descriptors)
    for c in range(numa):
        nd = sysfs / f"devices/system/node/node{c}"
        _w(nd / "meminfo", f"Node {c} MemTotal:       1048576 kB\n")
        _w(nd / "distance", " ".join("10" if i == c else "32" for i in range(numa)) + "\n")
        _w(nd / "cpulist", f"{c * spec.cpus_per_numa}-{(c + 1) * spec.cpus_per_numa - 1}\n")
        for k in range(spec.cpu_dirs_per_numa):
            cpu = c * spec.cpus_per_numa + k
            cd = sysfs / f"devices/system/cpu/cpu{cpu}"
            _w(cd / "online", "1\n")
            for idx, (lvl, typ, size) in enumerate([(1, "Data", "48K"), (1, "Instruction", "32K"), (2, "Unified", "1024K"),
                                                    (3, "Unified", "32768K")]):
                _w(cd / f"cache/index{idx}/level", f"{lvl}\n")
                _w(cd / f"cache/index{idx}/type", f"{typ}\n")
                _w(cd / f"cache/index{idx}/size", f"{size}\n")
            _link(sysfs / f"devices/system/cpu/cpu{cpu}", nd / f"cpu{cpu}")
    _w(sysfs / "devices/system/node/online", f"0-{numa - 1}\n")
    # CPU nodes 0..numa-1 (passthrough hosts run gim/vfio-pci, not amdgpu+kfd)
    for c in range(numa if spec.mode == "container" else 0):
        nd = nodes_dir / str(c)
        _w(nd / "properties", _props([
            ("cpu_cores_count", 64), ("simd_count", 0), ("mem_banks_count", 1), ("caches_count", 0),
            ("io_links_count", 0), ("p2p_links_count", 0), ("cpu_core_id_base", 64 * c), ("simd_id_base", 0),
            ("max_waves_per_simd", 0), ("lds_size_in_kb", 0), ("gds_size_in_kb", 0), ("num_gws", 0),
            ("wave_front_size", 0), ("array_count", 0), ("simd_arrays_per_engine", 0), ("cu_per_simd_array", 0),
            ("simd_per_cu", 0), ("max_slots_scratch_cu", 0), ("gfx_target_version", 0), ("vendor_id", 0),
            ("device_id", 0), ("location_id", 0), ("domain", 0), ("drm_render_minor", 0), ("hive_id", 0),
            ("num_sdma_engines", 0), ("num_sdma_xgmi_engines", 0), ("num_sdma_queues_per_engine", 0),
            ("num_cp_queues", 0), ("max_engine_clk_ccompute", 3700), ("local_mem_size", 0)]))
        _w(nd / "name", "")
        _w(nd / "gpu_id", "0")

    gpu_compute = spec.per_gpu_compute or [spec.compute_partition] * spec.num_gpus
    gpu_nodes: List[dict] = []
    node_id = numa
    render = 128
    card = 1
    xcp_counter = 0
    for g in range(spec.num_gpus):
        cp = gpu_compute[g].lower()
        parts = PARTITIONS[cp]
        bus = DEFAULT_BUSES[g] if g < len(DEFAULT_BUSES) else (0x10 + 8 * g) & 0xFF
        bdf = f"0000:{bus:02x}:00.0"
        uid = _unique_id(g)
        hive = _hive_id(g // max(1, spec.hive_size)) if spec.hive_size > 0 else 0
        numa_node = g * numa // spec.num_gpus
        info.bdfs.append(bdf)
        info.unique_ids.append(uid)
        info.hive_ids.append(hive)
        dev_dir = pci_root / bdf
        _w(dev_dir / "vendor", "0x1002")
        _w(dev_dir / "device", f"0x{spec.device_id:04x}")
        _w(dev_dir / "numa_node", str(numa_node))
        per = max(1, spec.cpus_per_numa)
        _w(dev_dir / "local_cpulist", f"{numa_node * per}-{numa_node * per + per - 1}")
        _w(dev_dir / "product_name", spec.product_name)
        # identity attributes amdgpu exposes on the PCI device (readable without
        # device-cgroup access, unlike kfd nodes): unique_id in hex, the hive id
        # in decimal, as on the MI355X box
        _w(dev_dir / "unique_id", f"{int(uid):016x}")
        _w(dev_dir / "mem_info_vram_total", str(MI355X_VRAM))
        if hive:
            _w(dev_dir / "xgmi_hive_info" / "xgmi_hive_id", str(hive))
        if spec.partition_support:
            _w(dev_dir / "current_compute_partition", cp.upper())
            _w(dev_dir / "current_memory_partition", spec.memory_partition.upper())
            _w(dev_dir / "available_compute_partition", "SPX, DPX, QPX, CPX")
            _w(dev_dir / "available_memory_partition", "NPS1, NPS2")
        iommu = sysfs / "kernel/iommu_groups" / str(10 + g)
        iommu.mkdir(parents=True, exist_ok=True)
        _link(iommu, dev_dir / "iommu_group")
        if spec.mode == "container":
            _link(drv_amdgpu, dev_dir / "driver")
            _link(dev_dir, drv_amdgpu / bdf)
        _link(dev_dir, sysfs / "bus/pci/devices" / bdf)
        kernel = spec.xcp_layout == "kernel"
        slots = 8 if kernel else parts
        if kernel:
            rank = (spec.probe_order or list(range(spec.num_gpus))).index(g)
            card, render = 8 * rank, 128 + 8 * rank
        for p in range(slots):
            if spec.mode != "container":
                break
            if p == 0:
                owner = dev_dir
                dev_name = bdf
            else:
                xcp_idx = 7 * rank + p - 1 if kernel else 8 * g + p
                owner = sysfs / "devices/platform" / f"amdgpu_xcp_{xcp_idx}"
                dev_name = f"amdgpu_xcp_{xcp_idx}"
                xcp_counter += 1
            (owner / "drm" / f"card{card}").mkdir(parents=True, exist_ok=True)
            (owner / "drm" / f"renderD{render}").mkdir(parents=True, exist_ok=True)
            _link(owner, sysfs / "class/drm" / f"card{card}" / "device")
            _link(owner, sysfs / "class/drm" / f"renderD{render}" / "device")
            if p > 0:
                # the platform device is not a PCI function; labeller reads through it
                _w(owner / "vendor", "0x1002")
                _w(owner / "device", f"0x{spec.device_id:04x}")
                _w(owner / "product_name", spec.product_name)
                _link(drv_amdgpu, owner / "driver")
            _w(dev / "dri" / f"card{card}", "")
            _w(dev / "dri" / f"renderD{render}", "")
            if p < parts:  # an active partition: a kubelet device with a kfd node
                info.device_ids.append(dev_name)
                info.render_minors[dev_name] = render
                info.node_ids[dev_name] = node_id
                info.gpu_of[dev_name] = g
                gpu_nodes.append(dict(node=node_id, gpu=g, part=p, parts=parts, bus=bus, uid=uid, hive=hive,
                                      numa=numa_node, render=render))
                node_id += 1
            render += 1
            card += 1

    # kfd GPU nodes
    for n in gpu_nodes:
        nd = nodes_dir / str(n["node"])
        parts = n["parts"]
        xcc = MI355X_XCDS // parts
        io_links = [dict(type=2, to=n["numa"], weight=20, bw_min=0, bw_max=64000)]
        p2p_links = []
        for m in gpu_nodes:
            if m["node"] == n["node"]:
                continue
            if m["gpu"] == n["gpu"]:
                io_links.append(dict(type=11, to=m["node"], weight=13, bw_min=819200, bw_max=819200))
            elif m["hive"] == n["hive"] and n["hive"] != 0:
                io_links.append(dict(type=11, to=m["node"], weight=15, bw_min=MI355X.xgmi_link_mbps,
                                     bw_max=MI355X.xgmi_link_mbps))
            else:
                p2p_links.append(dict(type=2, to=m["node"], weight=72, bw_min=0, bw_max=0))
        vram = MI355X_VRAM // parts
        if spec.memory_partition.lower() == "nps2" and parts == 1:
            vram = MI355X_VRAM
        props = [
            ("cpu_cores_count", 0), ("simd_count", MI355X_CUS * 4 // parts), ("mem_banks_count", 1),
            ("caches_count", 0), ("io_links_count", len(io_links)), ("p2p_links_count", len(p2p_links)),
            ("cpu_core_id_base", 0), ("simd_id_base", 2147487744 + 8 * n["node"]), ("max_waves_per_simd", 8),
            ("lds_size_in_kb", 160), ("gds_size_in_kb", 0), ("num_gws", 64), ("wave_front_size", 64),
            ("array_count", 4 * xcc), ("simd_arrays_per_engine", 1), ("cu_per_simd_array", 8),
            ("simd_per_cu", 4), ("max_slots_scratch_cu", 32), ("gfx_target_version", spec.gfx_target_version),
            ("vendor_id", 4098), ("device_id", spec.device_id), ("location_id", (n["bus"] << 8) | n["part"]),
            ("domain", 0), ("drm_render_minor", n["render"]), ("hive_id", n["hive"]),
            ("num_sdma_engines", 2), ("num_sdma_xgmi_engines", 6 if n["hive"] else 0),
            ("num_sdma_queues_per_engine", 8), ("num_cp_queues", 24), ("max_engine_clk_fcompute", 2400),
            ("local_mem_size", 0), ("fw_version", 200), ("capability", 2893521536), ("debug_prop", 1511),
            ("sdma_fw_version", 24), ("unique_id", n["uid"]), ("num_xcc", xcc), ("max_engine_clk_ccompute", 3700)]
        _w(nd / "properties", _props(props))
        _w(nd / "name", "gfx950")
        _w(nd / "gpu_id", str(40000 + n["node"]))
        for i, l in enumerate(io_links):
            _w(nd / "io_links" / str(i) / "properties", _props([
                ("type", l["type"]), ("version_major", 0), ("version_minor", 0), ("node_from", n["node"]),
                ("node_to", l["to"]), ("weight", l["weight"]), ("min_latency", 0), ("max_latency", 0),
                ("min_bandwidth", l["bw_min"]), ("max_bandwidth", l["bw_max"]), ("recommended_transfer_size", 0),
                ("recommended_sdma_engine_id_mask", 3), ("flags", 1)]))
        for i, l in enumerate(p2p_links):
            _w(nd / "p2p_links" / str(i) / "properties", _props([
                ("type", l["type"]), ("version_major", 0), ("version_minor", 0), ("node_from", n["node"]),
                ("node_to", l["to"]), ("weight", l["weight"]), ("min_latency", 0), ("max_latency", 0),
                ("min_bandwidth", 0), ("max_bandwidth", 0), ("recommended_transfer_size", 0),
                ("recommended_sdma_engine_id_mask", 0), ("flags", 3)]))
        _w(nd / "mem_banks/0/properties", _props([
            ("heap_type", 1), ("size_in_bytes", vram), ("flags", 0), ("width", 8192), ("mem_clk_max", 1900)]))

    if spec.mode == "vf":
        drv_gim = sysfs / "bus/pci/drivers/gim"
        drv_gim.mkdir(parents=True, exist_ok=True)
        _w(sysfs / "module/gim/version", "8.1.0.K+ddfa1e2")
        _w(sysfs / "module/gim/srcversion", "F00DFACE0123456789ABCDE")
        dev_vfio = dev / "vfio"
        dev_vfio.mkdir(parents=True, exist_ok=True)
        _w(dev_vfio / "vfio", "")
        info.device_ids = []
        for g, bdf in enumerate(info.bdfs):
            pf_dir = pci_root / bdf
            _link(drv_gim, pf_dir / "driver")
            for v in range(spec.vfs_per_gpu):
                bus = int(bdf.split(":")[1], 16)
                vf_bdf = f"0000:{bus:02x}:02.{v}"
                vf_dir = pci_root / vf_bdf
                _w(vf_dir / "vendor", "0x1002")
                _w(vf_dir / "device", f"0x{MI355X_VF_DEVICE_ID:04x}")
                grp = 100 + g * spec.vfs_per_gpu + v
                iommu = sysfs / "kernel/iommu_groups" / str(grp)
                iommu.mkdir(parents=True, exist_ok=True)
                _link(iommu, vf_dir / "iommu_group")
                _link(vf_dir, pf_dir / f"virtfn{v}")
                _link(vf_dir, sysfs / "bus/pci/devices" / vf_bdf)
                _w(dev_vfio / str(grp), "")
                info.device_ids.append(str(grp))
    elif spec.mode == "pf":
        drv_vfio = sysfs / "bus/pci/drivers/vfio-pci"
        drv_vfio.mkdir(parents=True, exist_ok=True)
        dev_vfio = dev / "vfio"
        dev_vfio.mkdir(parents=True, exist_ok=True)
        _w(dev_vfio / "vfio", "")
        info.device_ids = []
        for g, bdf in enumerate(info.bdfs):
            _link(drv_vfio, pci_root / bdf / "driver")
            _w(dev_vfio / str(10 + g), "")
            info.device_ids.append(str(10 + g))
    return info



def deny_kfd_nodes(fi: FixtureInfo, node_ids) -> None:
    """Make kfd GPU nodes unreadable the way a device cgroup does: kfd then
    answers EPERM for every file under the node (properties, gpu_id, name,
    io_links, p2p_links, mem_banks; profiles/archive/sysfs_access_box.json). Tests run
    as root, which ignores permission bits, so each file becomes a directory:
    it still exists but cannot be read as a file."""
    nodes = fi.sysfs / "class/kfd/kfd/topology/nodes"
    for nid in node_ids:
        nd = nodes / str(nid)
        for f in list(nd.rglob("*")):
            if f.is_file() and not f.is_symlink():
                f.unlink()
                f.mkdir()
        if not (nd / "properties").exists():
            (nd / "properties").mkdir(parents=True)


def wrap_kfd_topology(topology_dir: os.PathLike, root: os.PathLike) -> FixtureInfo:
    """A node sysfs around a captured kfd topology (e.g. the reference's
    ``testdata/topology-parsing/topology``, which holds only
    ``class/kfd/kfd/topology``): the topology is copied as is and every GPU
    node gets the PCI function, drm card/render nodes and /dev entries that the
    plugin's discovery joins it with (through ``drm_render_minor``, as
    ``GetDevIdsFromTopology`` does, amdgpu.go:406-445). The BDF comes from the
    node's ``domain`` / ``location_id``; a node that repeats another's
    location (the reference fixture's node 2 "is a cp of 1") gets the next
    free bus number, since two PCI functions cannot share one."""
    import shutil
    src = Path(topology_dir)
    root = Path(root)
    sysfs, dev = root / "sys", root / "dev"
    info = FixtureInfo(root=root, sysfs=sysfs, dev=dev)
    topo = sysfs / "class/kfd/kfd/topology"
    shutil.copytree(src, topo)
    if not (topo / "generation_id").exists():
        _w(topo / "generation_id", "1")
    pci_root = sysfs / "devices/pci0000:00"
    drv = sysfs / "bus/pci/drivers/amdgpu"
    drv.mkdir(parents=True, exist_ok=True)
    _w(sysfs / "module/amdgpu/version", "capture")
    (sysfs / "module/amdgpu/drivers").mkdir(parents=True, exist_ok=True)
    _link(sysfs / "module/amdgpu", drv / "module")
    _link(drv, sysfs / "module/amdgpu/drivers/pci:amdgpu")
    (dev / "dri").mkdir(parents=True, exist_ok=True)
    _w(dev / "kfd", "")
    used = set()
    nodes = sorted((p for p in (topo / "nodes").iterdir() if p.name.isdigit()), key=lambda p: int(p.name))
    for nd in nodes:
        props = {}
        for line in (nd / "properties").read_text().splitlines():
            k, _, v = line.partition(" ")
            props[k] = v.strip()
        if int(props.get("simd_count", "0")) == 0:
            continue
        loc, dom = int(props.get("location_id", "0")), int(props.get("domain", "0"))
        bus, devfn = (loc >> 8) & 0xFF, loc & 0xFF
        while (dom, bus, devfn) in used:
            bus = (bus + 1) & 0xFF
        used.add((dom, bus, devfn))
        bdf = f"{dom:04x}:{bus:02x}:{devfn >> 3:02x}.{devfn & 7:x}"
        minor = int(props.get("drm_render_minor", "0"))
        card = minor - 128
        dev_dir = pci_root / bdf
        _w(dev_dir / "vendor", f"0x{int(props.get('vendor_id', '4098')):04x}")
        _w(dev_dir / "device", f"0x{int(props.get('device_id', '0')):04x}")
        _w(dev_dir / "numa_node", "0")
        _link(drv, dev_dir / "driver")
        _link(dev_dir, drv / bdf)
        _link(dev_dir, sysfs / "bus/pci/devices" / bdf)
        (dev_dir / "drm" / f"card{card}").mkdir(parents=True, exist_ok=True)
        (dev_dir / "drm" / f"renderD{minor}").mkdir(parents=True, exist_ok=True)
        _link(dev_dir, sysfs / "class/drm" / f"card{card}" / "device")
        _link(dev_dir, sysfs / "class/drm" / f"renderD{minor}" / "device")
        _w(dev / "dri" / f"card{card}", "")
        _w(dev / "dri" / f"renderD{minor}", "")
        info.bdfs.append(bdf)
        info.device_ids.append(bdf)
        info.render_minors[bdf] = minor
        info.node_ids[bdf] = int(nd.name)
    return info
