"""Probe: how the GPU box exposes GPU <-> NUMA topology (KFD sysfs, PCI sysfs, env, torch)."""
import glob
import json
import os

out = {"env": {k: v for k, v in os.environ.items() if "VISIBLE" in k or k.startswith(("ROCR", "HIP_", "HSA_"))},
       "affinity": sorted(os.sched_getaffinity(0))[:8] + ["..."], "n_affinity": len(os.sched_getaffinity(0)),
       "cpu_count": os.cpu_count()}
nodes = {}
for d in sorted(glob.glob("/sys/devices/system/node/node*")):
    try:
        nodes[os.path.basename(d)] = open(os.path.join(d, "cpulist")).read().strip()
    except OSError as e:
        nodes[os.path.basename(d)] = str(e)
out["numa_nodes"] = nodes
kfd = []
for d in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*"), key=lambda x: int(os.path.basename(x))):
    props = {}
    try:
        for line in open(os.path.join(d, "properties")):
            k, _, v = line.strip().partition(" ")
            if k in ("simd_count", "location_id", "domain", "drm_render_minor", "gpu_id", "cpu_cores_count",
                     "unique_id", "num_xcc", "vendor_id", "device_id"):
                props[k] = v
    except OSError as e:
        props["err"] = str(e)
    props["node"] = os.path.basename(d)
    kfd.append(props)
out["kfd_nodes"] = kfd
for p in kfd:
    if p.get("simd_count", "0") != "0" and "location_id" in p:
        loc, dom = int(p["location_id"]), int(p.get("domain", 0))
        bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}"
        p["bdf"] = bdf
        try:
            p["pci_numa_node"] = open(f"/sys/bus/pci/devices/{bdf}/numa_node").read().strip()
        except OSError as e:
            p["pci_numa_node"] = str(e)
        rm = p.get("drm_render_minor")
        if rm:
            p["render_accessible"] = os.access(f"/dev/dri/renderD{rm}", os.R_OK | os.W_OK)
import torch  # noqa: E402

out["device_count"] = torch.cuda.device_count()
props = []
for i in range(torch.cuda.device_count()):
    pr = torch.cuda.get_device_properties(i)
    props.append({"i": i, "pci_bus_id": pr.pci_bus_id, "pci_device_id": pr.pci_device_id,
                  "pci_domain_id": pr.pci_domain_id, "name": pr.name})
out["torch_devices"] = props
print(json.dumps(out, indent=1))
