import json, sys
d = json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/conv_bench.json"))
for name, row in d.items():
    cells = []
    for k, v in row.items():
        flag = "" if v["rel_err_vs_generic"] < 1e-6 else "!"
        cells.append(f"{k}:{v['tflops']:6.1f}{flag}")
    print(name.ljust(28), "  ".join(cells))
