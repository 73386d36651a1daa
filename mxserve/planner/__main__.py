from .planner import main

main()
