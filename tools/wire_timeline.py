"""Timeline of the last traced step of the shares-from-the-wire close (bench.py --workload
resnet18-secagg-state under rocprofv3 --kernel-trace --memory-copy-trace): how busy the H2D link is,
the gaps between DMAs, how much of the varint decode runs beside a DMA, what follows the share sum.

    python tools/wire_timeline.py <rocprofv3 output dir with run_*_trace.csv>/
"""
import csv, sys
T = sys.argv[1]
mc = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), 'H2D') for r in csv.DictReader(open(T + 'run_memory_copy_trace.csv'))]
kt = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].replace('pgh::(anonymous namespace)::', '').replace('void ', '')[:24])
      for r in csv.DictReader(open(T + 'run_kernel_trace.csv'))]
ev = sorted(mc + kt)
sec = [e for e in ev if e[2].startswith('k_secagg<')]
end = sec[-1][1]; start = sec[-2][1]
win = [e for e in ev if start <= e[0] <= end]
h2d = [e for e in win if e[2] == 'H2D']
dec = [e for e in win if e[2].startswith('k_varint')]
span = (h2d[-1][1] - h2d[0][0]) / 1e6; busy = sum(e[1] - e[0] for e in h2d) / 1e6
print(f'step {(end - start) / 1e6:.2f} ms; H2D span {span:.2f} ms busy {busy:.2f} ms; {len(h2d)} copies, {len(dec)} decodes')
gaps = [(h2d[i + 1][0] - h2d[i][1]) / 1e3 for i in range(len(h2d) - 1)]
print('gap sum', round(sum(g for g in gaps if g > 0) / 1e3, 2), 'ms; gaps>20us:', [round(g) for g in gaps if g > 20])
print('window start -> first H2D', round((h2d[0][0] - start) / 1e3), 'us; last H2D end -> secagg start', round((sec[-1][0] - h2d[-1][1]) / 1e3), 'us; secagg', round((sec[-1][1] - sec[-1][0]) / 1e3), 'us')
d = sorted((e[1] - e[0]) / 1e3 for e in h2d); print('H2D dur us min/med/max', round(d[0]), round(d[len(d) // 2]), round(d[-1]))
# overlap of decodes with H2D
ov = 0
for a, b, _ in dec:
    for x, y, _ in h2d:
        ov += max(0, min(b, y) - max(a, x))
print('decode time', round(sum(b - a for a, b, _ in dec) / 1e6, 2), 'ms, overlapped with H2D', round(ov / 1e6, 2), 'ms')
after = [e for e in ev if e[0] >= sec[-1][1]][:4]
for e in after: print(' after secagg:', e[2], 'start +', round((e[0] - sec[-1][1]) / 1e3), 'us dur', round((e[1] - e[0]) / 1e3), 'us')
