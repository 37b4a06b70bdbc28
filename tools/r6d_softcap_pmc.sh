set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6d}
mkdir -p $O
timeout -k 10 300 python -u tools/softcap_ab.py spatialvla_amd/libsvla.so diag/libsvla_sc_div.so diag/libsvla_sc_wpb6.so diag/libsvla_sc_u8.so diag/libsvla_sc_u2.so > $O/softcap_ab.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/softcap_prof.py 5 > $O/plain.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --kernel-trace -d /tmp/p1 -o p --output-format csv -- python3 tools/softcap_prof.py 2 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/p2 -o p --output-format csv -- python3 tools/softcap_prof.py 2 > $O/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/p3 -o p --output-format csv -- python3 tools/softcap_prof.py 2 > $O/p3.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d /tmp/p4 -o p --output-format csv -- python3 tools/softcap_prof.py 2 > $O/p4.log 2>&1 || exit 1
python tools/pmc_table.py /tmp/p1 /tmp/p2 /tmp/p3 /tmp/p4 > $O/pmc_table.txt 2>&1
cat $O/softcap_ab.txt; cat $O/plain.txt; grep -A30 softcap_rows $O/pmc_table.txt
