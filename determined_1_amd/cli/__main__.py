from determined_1_amd.cli.cli import main

if __name__ == "__main__":
    main()
