"""Host timeline of the asynchronous ZeRO-Offload update (SXE_OFFLOAD_TRACE=1
SXE_OFFLOAD_TRACE_FILE=<path>): per optimizer step and unit, when its gradient D2H had landed, when
the C++ update started / ended (ms after step() began), and when the next forward waited for it.
  python tools/offload_timeline.py gpurun_out/offload_trace.jsonl [step]"""
import json
import sys


def main():
    rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows) - 1
    r = rows[k]
    waits = {n: (a, b) for n, a, b in r["waits"]}
    print(f"step {k}: {len(r['units'])} units, {r['elems'] / 1e9:.2f} G fp32 elements")
    print("| unit | elements | D2H landed (ms) | C++ update (ms) | next forward waited (ms) |")
    print("|---|---:|---:|---:|---:|")
    for name, n, ta, tb, tc in r["units"]:
        w = waits.get(name)
        ws = f"{w[0] * 1e3:.0f} - {w[1] * 1e3:.0f}" if w else "-"
        print(f"| {name} | {n / 1e6:.0f} M | {tb * 1e3:.0f} | {tb * 1e3:.0f} - {tc * 1e3:.0f} | {ws} |")


if __name__ == "__main__":
    main()
