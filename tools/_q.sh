bash tools/gpu_steps.sh "shg|150|python tools/shape_prof.py" "shg2|150|python tools/shape_prof.py"
