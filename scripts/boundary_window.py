# kernel timeline around one visual_lin_kernel launch of a rocprofv3 kernel trace (from the box-plus before
# it to the landmark elimination after it): boundary_window.py run_kernel_trace.csv INDEX (e.g. -2)
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
ks=[(int(r['Start_Timestamp']),int(r['End_Timestamp']),r['Kernel_Name'].replace('viba::','').replace('void ','').replace('(anonymous namespace)::','')[:34],r['Queue_Id'],int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])) for r in rows]
ks.sort()
vl=[i for i,k in enumerate(ks) if k[2].startswith('visual_lin')]
i=vl[int(sys.argv[2])]
t0=ks[i][0]
j=i
while not ks[j][2].startswith('boxplus_points'): j-=1
while not ks[j][2].startswith('landmark_'):
    s,e,n,q,g=ks[j]; print(f"{(s-t0)/1e3:8.1f} {(e-t0)/1e3:8.1f} {(e-s)/1e3:7.1f} q{q} g{g:6d} {n}"); j+=1
