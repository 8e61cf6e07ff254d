#!/bin/bash
# Round 6: mode-B kernel stats, then the MFMA-busy / LDS counter passes for mode A and mode B.
set -o pipefail
bash tools/prof_modeB_stats.sh r06m > gpurun_out/r06m_stats.txt 2>&1 || { echo "modeB stats failed"; tail -20 gpurun_out/r06m_stats.txt; exit 1; }
bash tools/pmc_mfma.sh r06m_mfmaA --no-extras > gpurun_out/r06m_mfmaA.txt 2>&1 || { echo "pmc A failed"; tail -20 gpurun_out/r06m_mfmaA.txt; exit 1; }
bash tools/pmc_mfma.sh r06m_mfmaB --mode B --no-extras > gpurun_out/r06m_mfmaB.txt 2>&1 || { echo "pmc B failed"; tail -20 gpurun_out/r06m_mfmaB.txt; exit 1; }
# keep what travels back small: the per-dispatch counter CSVs are summarised in pmc_mfma.json
find gpurun_out/r06m_mfmaA gpurun_out/r06m_mfmaB -name '*.csv' -size +2M -exec gzip {} \;
du -sh gpurun_out
