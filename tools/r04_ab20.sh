# round 4: switches re-checked after the argument laundering: B0 HEAD | AEC cooperative AppendEntries receive (MR_AE_COOP) |
# RX4 four-slot earliest-message rescan (MR_RESCAN_X4) | LV -amdgpu-load-store-vectorizer=0
PTEST="test_scenario_bit_exact and (figure_8_unreliable_2c or figure_8_unreliable_crash or snapshot_install_unreliable_2d)" TESTS="figure_8_unreliable_2c figure_8_unreliable_crash snapshot_install_unreliable_2d" bash tools/ab.sh ab20 B0 AEC RX4 LV || exit 1
