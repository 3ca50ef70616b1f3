# round 4: AppendEntries receive batch size re-checked after the argument laundering freed registers: A4 HEAD (MR_AC 4) | A5 | A6 | A8
PTEST="test_scenario_bit_exact and (figure_8_unreliable_2c or figure_8_unreliable_crash or snapshot_install_unreliable_2d)" TESTS="figure_8_unreliable_2c figure_8_unreliable_crash snapshot_install_unreliable_2d" bash tools/ab.sh ab24 A4 A5 A6 A8 || exit 1
