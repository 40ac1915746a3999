#!/usr/bin/env perl
# Test helper for tests/test_perl_xs.py: drives the Perl side of the XS binding
# (perl/lib/Prgpu.pm) on a chunk given as JSON {reads, alns, params}.
#
#   perl_cns_helper.pl pack IN.json  -> {field: hex of the packed pr_cns_batch buffer}
#   perl_cns_helper.pl run  IN.json  -> [{id, status, seq, qual, trace, cigar, chim}] (GPU)
#   perl_cns_helper.pl mem  IN.json  -> {head, rec, batch}: Prgpu::mem (the bwa-proovread
#       mem output) with host seeding, and the SW results either injected from IN.json's
#       `sw` (the tests' CPU oracle; `batch` is then the hex of the task arrays handed to it)
#       or from sw_run on the GPU
#   perl_cns_helper.pl iter IN.json  -> {batch, res}: Prgpu::iteration (host seeding + iter_run on
#       the GPU), or with `inject` the batch it would hand to iter_run (CPU)
#   perl_cns_helper.pl mask IN.json  -> {params, masked, mcrs, stats}: Prgpu::mask_params, and
#       Prgpu::mask on the GPU when IN.json has reads
use strict;
use warnings;
use FindBin;
use lib "$FindBin::RealBin/../perl/lib";
use JSON::PP;
use Prgpu;

my ($mode, $file) = @ARGV;
open my $fh, '<', $file or die "$file: $!\n";
my $in = decode_json(do { local $/; <$fh> });
close $fh;
my $json = JSON::PP->new->canonical;

if ($mode eq 'pack') {
    my $b = Prgpu::pack_chunk($in->{reads}, $in->{alns});
    my %hex = map { $_ => ($_ eq 'n_lr' ? $b->{$_} : unpack('H*', $b->{$_})) } keys %$b;
    print $json->encode(\%hex), "\n";
} elsif ($mode eq 'run') {
    my $ctx = Prgpu::Context->new(0);
    my @res = Prgpu::run_chunk($ctx, $in->{params}, $in->{reads}, $in->{alns});
    for my $r (@res) { $r->{chim_lines} = [Prgpu::chim_lines($r)]; $r->{fastq} = $r->{status} ? '' : Prgpu::fastq($r) }
    print $json->encode(\@res), "\n";
} elsif ($mode eq 'mem') {
    my %batch_hex;
    my $ctx = $in->{sw} ? sub {
        my ($b) = @_;
        %batch_hex = map { $_ => ($_ eq 'n_task' ? $b->{$_} : unpack('H*', $b->{$_})) } keys %$b;
        return $in->{sw};
    } : Prgpu::Context->new(0);
    my ($head, $rec) = Prgpu::mem(ctx => $ctx, seed_opts => $in->{seed_opts}, sw_opts => $in->{sw_opts},
                                  b => $in->{b}, l => $in->{l}, threads => $in->{threads}, cl => $in->{cl},
                                  lr_names => $in->{lr_names}, lr_seqs => $in->{lr_seqs},
                                  sr_names => $in->{sr_names}, sr_seqs => $in->{sr_seqs},
                                  sr_quals => $in->{sr_quals});
    print $json->encode({head => $head, rec => $rec, batch => \%batch_hex}), "\n";
} elsif ($mode eq 'iter') {
    # inject: capture the batch handed to iter_run and return an all-failed output (CPU)
    my %batch_hex;
    my $n = @{$in->{lr_seqs}};
    my $ctx = $in->{inject} ? sub {
        my ($b) = @_;
        %batch_hex = map { $_ => ($_ eq 'n_task' ? $b->{$_} : unpack('H*', $b->{$_})) } keys %$b;
        return {map({ $_ => '' } qw(seq qual trace cigar chim kept)), out_off => pack('q<*', (0) x ($n + 1)),
                chim_off => pack('q<*', (0) x ($n + 1)), status => pack('l<*', (-1) x $n),
                map({ $_ => pack('l<*', (0) x $n) } qw(seq_len trace_len ncigar nchim))};
    } : Prgpu::Context->new(0);
    my @res = Prgpu::iteration(ctx => $ctx, seed_opts => $in->{seed_opts}, sw_opts => $in->{sw_opts},
                               params => $in->{params}, threads => 2, lr_ids => $in->{lr_ids},
                               lr_seqs => $in->{lr_seqs}, lr_quals => $in->{lr_quals}, sr_seqs => $in->{sr_seqs});
    print $json->encode({batch => \%batch_hex, res => \@res}), "\n";
} elsif ($mode eq 'mask') {
    my $p = Prgpu::mask_params($in->{hcr_mask}, $in->{min_sr_length});
    my ($masked, $mcrs, $st) = $in->{seqs}
        ? Prgpu::mask(Prgpu::Context->new(0), hcr_mask => $in->{hcr_mask}, min_sr_length => $in->{min_sr_length},
                      seqs => $in->{seqs}, quals => $in->{quals})
        : ([], [], []);
    print $json->encode({params => $p, masked => $masked, mcrs => $mcrs, stats => $st}), "\n";
} else {
    die "usage: perl_cns_helper.pl pack|run|mem|iter|mask IN.json\n";
}
