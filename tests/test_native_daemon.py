"""The native daemon (`mi355x-device-plugin`, native/src/daemon/): the device
plugin as one C++ process, driven end to end by the fake kubelet on generated
MI355X sysfs trees. Its ListAndWatch lists, GetPreferredAllocation and
Allocate answers must equal the Python plugin's (ContainerImpl) on the same
node; registration, kubelet restarts, exporter health and SIGTERM follow the
reference (cmd/k8s-device-plugin/main.go, vendored dpm manager/plugin)."""
import asyncio
import os
import random
import signal
import subprocess
import time

import pytest

from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
from rocm_k8s_device_plugin_amd.plugin.base import new_context
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
from rocm_k8s_device_plugin_amd.testing.fake_exporter import FakeExporter
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node

# MI355X_NATIVE_DAEMON_EXE: run these tests against another build (e.g. the ASan / TSan ctest builds)
EXE = os.environ.get("MI355X_NATIVE_DAEMON_EXE") or os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} was not built")


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


async def _daemon(kdir, fi, *extra):
    return await asyncio.create_subprocess_exec(
        EXE, "-kubelet_dir", kdir, "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), *extra,
        stdout=asyncio.subprocess.DEVNULL, stderr=asyncio.subprocess.PIPE)


async def _stop(proc):
    if proc.returncode is None:
        proc.send_signal(signal.SIGTERM)
    _, err = await asyncio.wait_for(proc.communicate(), 20)
    return proc.returncode, err.decode(errors="replace")


def _python_impl(fi, strategy="single"):
    return ContainerImpl(strategy, str(fi.sysfs), HealthConfig(exporter_socket=None))


@pytest.mark.parametrize("partition,strategy,resource", [("spx", "single", "gpu"), ("cpx", "single", "gpu"),
                                                         ("cpx", "mixed", "cpx_nps1")])
def test_answers_equal_the_python_plugin(tmp_path, partition, strategy, resource):
    fi = make_mi355x_node(tmp_path / "n", compute_partition=partition)
    impl = _python_impl(fi, strategy)
    ctx = new_context(resource)
    impl.start(ctx)
    kdir = str(tmp_path / "dp")

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        proc = await _daemon(kdir, fi, "-exporter_socket", "", "-resource_naming_strategy", strategy)
        try:
            st = await k.wait_for_resource(f"amd.com/{resource}", len(impl.devices(resource)), timeout=20)
            # the list kubelet received, device for device
            want = {d.ID: d.health for d in impl.enumerate(ctx)}
            assert st.devices == want
            opts = await k._call(st, "GetDevicePluginOptions", pb.Empty(), pb.DevicePluginOptions)
            assert opts == impl.options(ctx)
            rng = random.Random(3)
            ids = sorted(want)
            for _ in range(25):
                avail = sorted(rng.sample(ids, rng.randint(1, len(ids))))
                size = rng.randint(1, len(avail))
                must = sorted(rng.sample(avail, rng.randint(0, min(2, size))))
                preq = pb.PreferredAllocationRequest(container_requests=[pb.ContainerPreferredAllocationRequest(
                    available_deviceIDs=avail, must_include_deviceIDs=must, allocation_size=size)])
                got = await k._call(st, "GetPreferredAllocation", preq, pb.PreferredAllocationResponse)
                assert got == impl.preferred_allocation(ctx, preq)
                chosen = list(got.container_responses[0].deviceIDs)
                areq = pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(devices_ids=chosen),
                                                              pb.ContainerAllocateRequest(devices_ids=[])])
                assert await k._call(st, "Allocate", areq, pb.AllocateResponse) == impl.allocate(ctx, areq)
            pre = await k._call(st, "PreStartContainer", pb.PreStartContainerRequest(devices_ids=ids[:1]),
                                pb.PreStartContainerResponse)
            assert pre == pb.PreStartContainerResponse()
            reg = k.registrations[-1]
            assert (reg.version, reg.endpoint, reg.resource_name) == ("v1beta1", f"amd.com_{resource}",
                                                                      f"amd.com/{resource}")
            assert reg.options.get_preferred_allocation_available
        finally:
            rc, err = await _stop(proc)
            await k.stop()
        assert rc == 0, err[-2000:]
        assert not os.path.exists(os.path.join(kdir, f"amd.com_{resource}"))   # socket removed on SIGTERM

    run(go())


def test_unknown_device_id_is_invalid_argument(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        proc = await _daemon(kdir, fi, "-exporter_socket", "")
        try:
            st = await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            with pytest.raises(Exception) as ei:
                await k._call(st, "Allocate", pb.AllocateRequest(container_requests=[
                    pb.ContainerAllocateRequest(devices_ids=["nope"])]), pb.AllocateResponse)
            assert "unknown device ID 'nope'" in str(ei.value.details() if hasattr(ei.value, "details") else ei.value)
        finally:
            rc, err = await _stop(proc)
            await k.stop()
        assert rc == 0, err[-2000:]

    run(go())


def test_kubelet_restart_re_registers(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        proc = await _daemon(kdir, fi, "-exporter_socket", "")
        try:
            await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            first = k.register_times["amd.com/gpu"]
            t0 = time.monotonic()
            await k.restart(downtime_s=0.2)
            st = await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            assert k.register_times["amd.com/gpu"] > first
            assert k.register_times["amd.com/gpu"] - t0 < 2.0      # inotify, not a poll
            adm = await k.admit("amd.com/gpu", 2)
            assert len(adm.device_ids) == 2 and st.devices
        finally:
            rc, err = await _stop(proc)
            await k.stop()
        assert rc == 0, err[-2000:]

    run(go())


def test_exporter_verdict_reaches_listandwatch(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")
    sock = str(tmp_path / "exp" / "exporter.sock")

    async def go():
        exp = FakeExporter(sock, {b: "healthy" for b in fi.bdfs})
        await exp.start()
        k = FakeKubelet(kdir)
        await k.start()
        proc = await _daemon(kdir, fi, "-exporter_socket", sock, "-pulse", "1")
        try:
            st = await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            assert all(h == "Healthy" for h in st.devices.values())
            u = st.updates
            exp.states[fi.bdfs[5]] = "unhealthy"
            st = await k.wait_for_update("amd.com/gpu", u, timeout=10)
            assert st.devices[fi.bdfs[5]] == "Unhealthy"
            assert sum(h == "Unhealthy" for h in st.devices.values()) == 1
            exp.states[fi.bdfs[5]] = "healthy"
            st = await k.wait_for_update("amd.com/gpu", st.updates, timeout=10)
            assert all(h == "Healthy" for h in st.devices.values())
        finally:
            rc, err = await _stop(proc)
            await k.stop()
            await exp.stop()
        assert rc == 0, err[-2000:]

    run(go())


def test_exporter_verdict_covers_every_partition_of_the_gpu(tmp_path):
    """CPX: the exporter's per-BDF verdict marks all 8 partitions of that GPU."""
    fi = make_mi355x_node(tmp_path / "n", compute_partition="cpx")
    kdir = str(tmp_path / "dp")
    sock = str(tmp_path / "exp" / "exporter.sock")
    impl = _python_impl(fi)
    parts = [d.id for d in impl.inv.devices if d.bdf == fi.bdfs[3]]
    assert len(parts) == 8

    async def go():
        exp = FakeExporter(sock, {b: "healthy" for b in fi.bdfs})
        await exp.start()
        k = FakeKubelet(kdir)
        await k.start()
        proc = await _daemon(kdir, fi, "-exporter_socket", sock, "-pulse", "1")
        try:
            st = await k.wait_for_resource("amd.com/gpu", 64, timeout=20)
            exp.states[fi.bdfs[3]] = "unhealthy"
            st = await k.wait_for_update("amd.com/gpu", st.updates, timeout=10)
            assert sorted(i for i, h in st.devices.items() if h == "Unhealthy") == sorted(parts)
        finally:
            rc, err = await _stop(proc)
            await k.stop()
            await exp.stop()
        assert rc == 0, err[-2000:]

    run(go())


def test_kfd_node_loss_marks_the_device_unhealthy(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        proc = await _daemon(kdir, fi, "-exporter_socket", "", "-pulse", "1")
        try:
            st = await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            impl = _python_impl(fi)
            dev = impl.inv.by_id[fi.bdfs[2]]
            os.unlink(fi.sysfs / f"class/kfd/kfd/topology/nodes/{dev.node_id}/properties")
            st = await k.wait_for_update("amd.com/gpu", st.updates, timeout=10)
            assert st.devices[fi.bdfs[2]] == "Unhealthy"
        finally:
            rc, err = await _stop(proc)
            await k.stop()
        assert rc == 0, err[-2000:]

    run(go())


def test_starts_before_the_kubelet_and_registers_when_it_comes(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    kdir = str(tmp_path / "dp")
    os.makedirs(kdir)

    async def go():
        proc = await _daemon(kdir, fi, "-exporter_socket", "")
        await asyncio.sleep(0.5)
        k = FakeKubelet(kdir)
        await k.start()
        try:
            await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
        finally:
            rc, err = await _stop(proc)
            await k.stop()
        assert rc == 0, err[-2000:]

    run(go())


def test_flags(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    base = [EXE, "-kubelet_dir", str(tmp_path / "dp"), "-sysfs_root", str(fi.sysfs)]
    p = subprocess.run(base + ["-driver_type", "gpu"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 1 and "invalid driver_type provided: gpu" in p.stderr
    p = subprocess.run(base + ["-resource_naming_strategy", "x"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 1 and "invalid resource_naming_strategy" in p.stderr
    p = subprocess.run(base + ["-pulse=-1"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 1 and "pulse must be a non-negative integer" in p.stderr
    # an explicitly requested driver that cannot start exits 1 (main.go:94-105)
    p = subprocess.run(base + ["-driver_type=vf-passthrough"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 1 and "No amd gim driver loaded" in p.stderr
    p = subprocess.run(base + ["-driver_type=pf-passthrough"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 1 and "No vfio-pci driver loaded" in p.stderr
    p = subprocess.run([EXE, "-h"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 0 and "-resource_naming_strategy" in p.stdout
    # heterogeneous partitions with the single strategy: the reference's init error
    het = make_mi355x_node(tmp_path / "het", per_gpu_compute=["spx"] * 4 + ["cpx"] * 4)
    p = subprocess.run([EXE, "-kubelet_dir", str(tmp_path / "dp2"), "-sysfs_root", str(het.sysfs), "-driver_type",
                        "container"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 1 and "not supported with single strategy" in p.stderr
    # without -driver_type the next implementations are tried, and with none the daemon idles (main.go:106-119)
    q = subprocess.Popen([EXE, "-kubelet_dir", str(tmp_path / "dp3"), "-sysfs_root", str(het.sysfs)],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    time.sleep(0.5)
    q.send_signal(signal.SIGTERM)
    _, err = q.communicate(timeout=20)
    assert q.returncode == 0 and "not supported with single strategy" in err and "No vfio-pci driver loaded" in err


@pytest.mark.gpu
def test_real_node_answers_equal_the_python_plugin(tmp_path):
    """On the MI355X box's own /sys (where kfd denies the GPUs outside this
    container's cgroup): the same devices, health, options and Allocate answers
    as the Python plugin."""
    impl = ContainerImpl("single", "/sys", HealthConfig(exporter_socket=None))
    ctx = new_context("gpu")
    impl.start(ctx)
    want = {d.ID: d.health for d in impl.enumerate(ctx)}
    assert want, "no GPUs discovered on the box"
    kdir = str(tmp_path / "dp")

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        t0 = time.monotonic()
        proc = await asyncio.create_subprocess_exec(EXE, "-kubelet_dir", kdir, "-exporter_socket", "", "-pulse", "1",
                                                    stdout=asyncio.subprocess.DEVNULL, stderr=asyncio.subprocess.PIPE)
        try:
            st = await k.wait_for_resource("amd.com/gpu", len(want), timeout=20)
            registered_s = k.register_times["amd.com/gpu"] - t0
            assert st.devices == want
            assert await k._call(st, "GetDevicePluginOptions", pb.Empty(), pb.DevicePluginOptions) == impl.options(ctx)
            ids = sorted(want)
            for size in sorted({1, min(2, len(ids)), len(ids)}):
                preq = pb.PreferredAllocationRequest(container_requests=[pb.ContainerPreferredAllocationRequest(
                    available_deviceIDs=ids, allocation_size=size)])
                got = await k._call(st, "GetPreferredAllocation", preq, pb.PreferredAllocationResponse)
                assert got == impl.preferred_allocation(ctx, preq)
                areq = pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(
                    devices_ids=list(got.container_responses[0].deviceIDs))])
                assert await k._call(st, "Allocate", areq, pb.AllocateResponse) == impl.allocate(ctx, areq)
            await asyncio.sleep(1.5)     # a health pulse on the live kfd nodes changes nothing
            assert k.resources["amd.com/gpu"].devices == want
        finally:
            rc, err = await _stop(proc)
            await k.stop()
        assert rc == 0, err[-2000:]
        print(f"native daemon on the box: {len(want)} devices, registered {registered_s * 1e3:.1f} ms after exec")

    run(go())


def _passthrough_impl(fi, mode, strategy):
    from rocm_k8s_device_plugin_amd.plugin.passthrough import PfImpl, VfImpl
    cls = VfImpl if mode == "vf" else PfImpl
    return cls(strategy, str(fi.sysfs), exporter_socket=None)


@pytest.mark.parametrize("mode,strategy,resource", [("vf", "single", "gpu"), ("vf", "mixed", "gpu_vf"),
                                                    ("pf", "single", "gpu"), ("pf", "mixed", "gpu_pf")])
def test_passthrough_answers_equal_the_python_plugin(tmp_path, mode, strategy, resource):
    """VF / PF passthrough (amdgpu_sriov.go, amdgpu_pf.go), picked by the
    container -> VF -> PF auto-selection: one device per IOMMU group, Allocate
    with the vfio nodes and PCI_RESOURCE_AMD_COM_<RES> listing every requested
    group's BDFs, no preferred allocation; answers equal the Python impls'."""
    fi = make_mi355x_node(tmp_path / "n", mode=mode, vfs_per_gpu=2)
    impl = _passthrough_impl(fi, mode, strategy)
    ctx = new_context(resource)
    impl.start(ctx)
    kdir = str(tmp_path / "dp")

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        proc = await _daemon(kdir, fi, "-exporter_socket", "", "-resource_naming_strategy", strategy)
        try:
            want = {d.ID: d.health for d in impl.enumerate(ctx)}
            st = await k.wait_for_resource(f"amd.com/{resource}", len(want), timeout=20)
            assert st.devices == want and len(want) == (16 if mode == "vf" else 8)
            opts = await k._call(st, "GetDevicePluginOptions", pb.Empty(), pb.DevicePluginOptions)
            assert opts == impl.options(ctx) and not opts.get_preferred_allocation_available
            ids = sorted(want)
            rng = random.Random(5)
            for _ in range(10):
                pick = rng.sample(ids, rng.randint(1, 4))
                areq = pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(devices_ids=pick),
                                                              pb.ContainerAllocateRequest(devices_ids=[])])
                got = await k._call(st, "Allocate", areq, pb.AllocateResponse)
                assert got == impl.allocate(ctx, areq)
                env = got.container_responses[0].envs[f"PCI_RESOURCE_AMD_COM_{resource.upper()}"]
                assert len(env.split(",")) == len(pick)   # one function per group in these trees
            preq = pb.PreferredAllocationRequest(container_requests=[pb.ContainerPreferredAllocationRequest(
                available_deviceIDs=ids, allocation_size=1)])
            assert await k._call(st, "GetPreferredAllocation", preq, pb.PreferredAllocationResponse) == \
                pb.PreferredAllocationResponse()
        finally:
            rc, err = await _stop(proc)
            await k.stop()
        assert rc == 0, err[-2000:]

    run(go())


def test_vf_health_follows_gim_and_the_exporter(tmp_path):
    """A VF group is Unhealthy when its parent PF is (exporter), and every group
    when the gim driver goes away (amdgpu_sriov.go:217-308)."""
    import shutil
    fi = make_mi355x_node(tmp_path / "n", mode="vf", vfs_per_gpu=2)
    impl = _passthrough_impl(fi, "vf", "single")
    kdir = str(tmp_path / "dp")
    sock = str(tmp_path / "exp" / "exporter.sock")
    bad_pf = fi.bdfs[2]
    bad_groups = sorted(g for g, fns in impl.groups.items() if any(f.pf == bad_pf for f in fns))
    assert len(bad_groups) == 2

    async def go():
        exp = FakeExporter(sock, {b: "healthy" for b in fi.bdfs})
        await exp.start()
        k = FakeKubelet(kdir)
        await k.start()
        proc = await _daemon(kdir, fi, "-exporter_socket", sock, "-pulse", "1", "-driver_type", "vf-passthrough")
        try:
            st = await k.wait_for_resource("amd.com/gpu", 16, timeout=20)
            assert set(st.devices.values()) == {"Healthy"}
            exp.states[bad_pf] = "unhealthy"
            st = await k.wait_for_update("amd.com/gpu", st.updates, timeout=10)
            assert sorted(i for i, h in st.devices.items() if h == "Unhealthy") == bad_groups
            shutil.rmtree(fi.sysfs / "bus/pci/drivers/gim")
            st = await k.wait_for_update("amd.com/gpu", st.updates, timeout=10)
            assert set(st.devices.values()) == {"Unhealthy"}
        finally:
            rc, err = await _stop(proc)
            await k.stop()
            await exp.stop()
        assert rc == 0, err[-2000:]

    run(go())
