import csv,glob,sys
for d in sys.argv[1:]:
    f=glob.glob(d+'/**/run_kernel_trace.csv',recursive=True)[0]
    rows=sorted((int(r['Start_Timestamp']),int(r['End_Timestamp'])) for r in csv.DictReader(open(f)) if 'mh_kernel' in r['Kernel_Name'])
    print(d, ' '.join('%.3f'%((e-s)/1e6) for s,e in rows))
    print('   gaps', ' '.join('%.3f'%((rows[i+1][0]-rows[i][1])/1e6) for i in range(len(rows)-1)))
