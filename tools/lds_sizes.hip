// Prints the LDS footprint of each stage of the encoder / decoder workspaces (build-time check).
#include <cstdio>
#include <cstddef>
#include "../rawnanoporesignalcompression_amd/csrc/pgn_zenc.h"
#include "../rawnanoporesignalcompression_amd/csrc/pgn_zdec.h"
using namespace pgn;
int main()
{
    EncLds* e = nullptr;
    printf("EncLds %zu\n", sizeof(EncLds));
    printf("  search filt+v %zu\n", sizeof(e->filt) + sizeof(e->vh0) * 3);
    printf("  lit hist2 %zu count %zu nbBits %zu val %zu nodes %zu tanc %zu tdep %zu win %zu hdr-set %zu\n", sizeof(e->hist2),
           sizeof(e->count), sizeof(e->nbBits), sizeof(e->val), sizeof(e->nodes), sizeof(e->tanc), sizeof(e->tdep),
           sizeof(e->win), sizeof(e->weights) + sizeof(e->hdr) + sizeof(e->fct) + sizeof(e->fscratch) + sizeof(e->wcount) + sizeof(e->wnorm) + sizeof(e->wcumul));
    printf("  seq sct %zu stsym %zu rest %zu\n", sizeof(e->sct), sizeof(e->stsym),
           sizeof(e->scount) + sizeof(e->snorm) + sizeof(e->scumul) + sizeof(e->snc) + sizeof(e->sv) + sizeof(e->sc));
    DecLds* d = nullptr;
    printf("DecLds %zu\n", sizeof(DecLds));
    printf("  lit tab %zu bmp %zu stg %zu wts %zu order %zu hbuf %zu wdt %zu\n", sizeof(d->tab), sizeof(d->bmp),
           sizeof(d->stg), sizeof(d->wts), sizeof(d->order), sizeof(d->hbuf), sizeof(d->wdt));
    printf("  seq qtab %zu qnorm %zu qsq %zu qhdr %zu qwin %zu\n", sizeof(d->qtab), sizeof(d->qnorm), sizeof(d->qsq),
           sizeof(d->qhdr), sizeof(d->qwin));
    return 0;
}
