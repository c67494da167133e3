"""Print the kernels of the LAST training step of a rocprofv3 kernel trace, in launch order,
with duration and grid; optional substring filter.  Step boundary = normalize_image_kernel."""
import csv
import re
import sys

path = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ''
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
starts = [i for i, r in enumerate(rows) if 'normalize_image' in r['Kernel_Name']]
step = rows[starts[-1]:] if starts else rows
tot = 0.0
for r in step:
    name = r['Kernel_Name']
    m = re.search(r'rod::(\w+)', name) or re.search(r'_ZN3rod\d+(\w+?)I', name) or re.search(r'(\w+)\(', name)
    short = m.group(1) if m else name[:40]
    dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    tot += dur
    if filt and filt not in name:
        continue
    grid = f"{int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
    print(f"{dur:9.1f}us  {short[:34]:34s} grid={grid:16s} vgpr={r['VGPR_Count']:>3s} lds={r['LDS_Block_Size']}")
print(f'step kernel total {tot/1e3:.3f} ms, {len(step)} kernels')
