mkdir -p gpurun_out
export DLA_HOST_REDUCE_STATS=1
python -c "import torch; p=torch.cuda.get_device_properties(0); print(p.pci_bus_id, p.pci_device_id, getattr(p,'pci_domain_id',None))" > gpurun_out/r02zb_pci.log 2>&1
for i in 1 2 3; do for b in none gpu; do
  PROBE_BIND=$b timeout -k 10 200 python profiles/host_reduce_probe.py "ns,configs[3'],configs[4]" > gpurun_out/r02zb_probe_${b}_$i.log 2>&1 || exit 1
done; done
