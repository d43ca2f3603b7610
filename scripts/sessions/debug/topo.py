import glob, os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
for d in sorted(glob.glob("/sys/bus/pci/devices/*")):
    try:
        vendor = open(d + "/vendor").read().strip()
        cls = open(d + "/class").read().strip()
    except Exception:
        continue
    if vendor == "0x1002" and cls.startswith("0x12"):
        print(os.path.basename(d), "numa", open(d + "/numa_node").read().strip(), "cpus", open(d + "/local_cpulist").read().strip())
l3 = set()
for c in sorted(glob.glob("/sys/devices/system/cpu/cpu[0-9]*"), key=lambda p: int(p.split("cpu")[-1])):
    try:
        l3.add(open(c + "/cache/index3/shared_cpu_list").read().strip())
    except Exception:
        pass
print("L3 groups", len(l3), sorted(l3, key=lambda s: int(s.split("-")[0].split(",")[0]))[:6])
print("affinity", sorted(os.sched_getaffinity(0))[:8], len(os.sched_getaffinity(0)))
import torch
p = torch.cuda.get_device_properties(0)
print("torch props", {k: getattr(p, k) for k in dir(p) if "pci" in k})
print("visible", os.environ.get("HIP_VISIBLE_DEVICES"), os.environ.get("ROCR_VISIBLE_DEVICES"), os.environ.get("CUDA_VISIBLE_DEVICES"))
