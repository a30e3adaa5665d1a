import sys, json, torch
sys.path.insert(0, '.')
import bench
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
stream = torch.cuda.current_stream(dev)
for ns in [int(x) for x in sys.argv[1].split(',')]:
    bench.LOG_STREAMS = ns
    for n in (1 << 20, 1 << 22):
        line = bench.log_faulty_line(stream, dev, n=n, general=False)
        print(json.dumps({"streams": ns, "n": n, "instances_per_s": line["instances_per_s"], "kernel_ms": line["kernel_ms"]}), flush=True)
